"""Host-side pieces of bench.py that need no GPU: the CPU baselines (oracle timed on this
host, single process and pooled) and the PMC-traffic lookup the roofline object uses."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _args(**kw):
    import argparse
    a = dict(size=64, kind="ct12", payload_chars=8, pee_T=2, cpu_seconds=0.05, cpu_ref_seconds=0.05, cpu_pool=2)
    a.update(kw)
    return argparse.Namespace(**a)


def test_cpu_baseline_small():
    r = bench.cpu_baseline(_args())
    assert r["kind"] == "port" and r["cores"] == 1 and r["value"] > 0 and r["unit"] == "Mpixels/s"
    assert "pee_cpu" in r["sample"] and r["reference_path"]["value"] > 0
    assert "reference_path" not in bench.cpu_baseline(_args(cpu_ref_seconds=0))


def test_cpu_baseline_pool_small():
    for which in ("pee", "lsb"):
        r = bench.cpu_baseline_pool(_args(), which, per_worker=1)
        assert r["cores"] == 2 and r["value"] > 0 and "pool" in r["sample"] and which in r["sample"]


def test_payload_equal_masks_lengths():
    import numpy as np
    import torch
    want = torch.from_numpy(np.array([[0b1011, 0], [-1, -1]], dtype=np.int64))
    got = want.clone()
    assert bench.payload_equal(got, want, [4, 128])
    got[0, 0] = 0b0011                       # a recovered bit differs
    assert not bench.payload_equal(got, want, [4, 128])
    got[0, 0] = 0b1011 | (1 << 9)            # a bit set past the slice's length
    assert not bench.payload_equal(got, want, [4, 128])
    assert bench.payload_equal(want, torch.from_numpy(np.array([[0b1011 | (1 << 9), 0], [-1, -1]])), [4, 128])


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
    # template-argument selection (argument 2 = INPLACE of the PEE kernels)
    assert bench.pmc_traffic("k_pee_embed1", 4, 8, 8, "ct12", {2: "true"})["hbm_bytes_per_launch"] == 2
    r = bench.pmc_traffic("k_pee_embed1", 4, 8, 8, "ct12", {2: "false"})
    assert r["hbm_bytes_per_launch"] == 1 and r["instance"] == "k_pee_embed1<unsigned short, true, false>"
    assert bench.pmc_traffic("k_pee_embed1", 4, 8, 8, "ct12", {5: "true"}) is None


def test_committed_pmc_summaries_resolve_every_bench_instance():
    """The roofline objects of the headline, in-place and C3 legs find their PMC rows in the
    committed summaries (the in-place lookup never matched)."""
    for tag, ta in (("k_pee_embed1", {2: "false"}), ("k_pee_extract1", {2: "false"}),
                    ("k_pee_embed_ss", {2: "true", 5: "false"}), ("k_pee_extract_ss", {2: "true"})):
        assert bench.pmc_traffic(tag, 256, 2048, 2048, "ct12", ta) is not None, tag
    for tag, ta in (("k_pee_embed_res", {}), ("k_pee_extract_ss", {2: "false"})):   # C3 (round 3 kernels)
        assert bench.pmc_traffic(tag, 256, 512, 512, "ct12", ta) is not None, tag


def test_gpus_world_size_mismatch_is_refused():
    """bench.py --gpus N under a launcher that started a different number of ranks exits
    non-zero before touching the GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
