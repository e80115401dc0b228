"""Host-side pieces of bench.py that need no GPU: the CPU baselines (oracle timed on this
host, single process and pooled) and the PMC-traffic lookup the roofline object uses."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_cpu_baseline_small():
    r = bench.cpu_baseline(64, "ct12", 8, 0.05)
    assert r["kind"] == "port" and r["cores"] == 1 and r["value"] > 0 and r["unit"] == "Mpixels/s"


def test_cpu_baseline_pool_small():
    r = bench.cpu_baseline_pool(64, "ct12", 8, 2, 1)
    assert r["cores"] == 2 and r["value"] > 0 and "pool" in r["sample"]


def test_pmc_traffic_lookup(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    d = {"config": {"batch": 4, "h": 8, "w": 8, "kind": "ct12"}, "source": "x",
         "kernels": {"k_scan_rows<unsigned short, 16, true, true, 0, true>": {"hbm_bytes_per_launch": 123},
                     "k_pee_embed1<unsigned short, true, false>": {"hbm_bytes_per_launch": 1},
                     "k_pee_embed1<unsigned short, true, true>": {"hbm_bytes_per_launch": 2}}}
    (prof / "pmc_traffic.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.pmc_traffic("k_scan_rows", 4, 8, 8, "ct12")["hbm_bytes_per_launch"] == 123
    assert bench.pmc_traffic("k_pee_embed1", 4, 8, 8, "ct12") is None      # ambiguous instantiation
    assert bench.pmc_traffic("k_scan_rows", 8, 8, 8, "ct12") is None       # other configuration
