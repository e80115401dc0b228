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
    assert r["pinned_core"] == min(os.sched_getaffinity(0)) and r["cores_available"] == len(os.sched_getaffinity(0))
    assert "pee_cpu" in r["sample"] and r["reference_path"]["value"] > 0
    assert "reference_path" not in bench.cpu_baseline(_args(cpu_ref_seconds=0))


def test_cpu_baseline_pool_small():
    for which in ("pee", "lsb"):
        r = bench.cpu_baseline_pool(_args(), which, per_worker=1)
        assert r["cores"] == 2 and r["value"] > 0 and "pool" in r["sample"] and which in r["sample"]
        assert r["pinned_cores"] == sorted(os.sched_getaffinity(0))[:2]
    # the pool never exceeds the cores this process may use
    big = bench.cpu_baseline_pool(_args(cpu_pool=10_000), "pee", per_worker=1)
    assert big["cores"] == len(os.sched_getaffinity(0)) == big["cores_available"]


def test_pinned_workers_run_on_their_core():
    cores = sorted(os.sched_getaffinity(0))[:2]
    with bench._pinned_pool(2, cores) as pool:
        got = sorted(pool.map(_affinity_of_worker, range(8), chunksize=1))
    assert set(got) <= {frozenset([c]) for c in cores}


def _affinity_of_worker(_i):
    import time
    time.sleep(0.05)
    return frozenset(os.sched_getaffinity(0))


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
    for tag, ta in (("k_pee_embed_res", {}), ("k_pee_extract_ss", {2: "false"}), ("k_scan_decide", {}),
                    ("k_restore_il", {})):   # C3
        assert bench.pmc_traffic(tag, 256, 512, 512, "ct12", ta) is not None, tag
    for tag, ta in (("k_pee_embed1", {2: "false"}), ("k_pee_extract1", {2: "false"}), ("k_scan_fast", {})):   # C2
        assert bench.pmc_traffic(tag, 1, 2048, 2048, "ct12", ta) is not None, tag
    # every source is this round's
    for tag, shape in (("k_pee_embed1", (256, 2048, 2048)), ("k_scan_decide", (256, 512, 512)), ("k_scan_fast", (1, 2048, 2048))):
        assert "profiles/r06/" in bench.pmc_traffic(tag, *shape, "ct12", {2: "false"} if tag == "k_pee_embed1" else {})["source"]


def _launcher(env_extra):
    """bench.py --gpus 2 --backend gloo without a launcher, ranks driven by the fault knobs
    (they act right after init_process_group, before any GPU call, so this runs on CPU)."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo", "--cpu-seconds", "0"]
    return subprocess.Popen(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def _rank_pids(proc, timeout=120):
    """Read the launcher's stderr until it names its rank pids."""
    import time
    t0 = time.monotonic()
    seen = []
    for line in proc.stderr:
        seen.append(line)
        if line.startswith("bench.py: rank pids "):
            return [int(x) for x in line.split()[3:]], seen
        assert time.monotonic() - t0 < timeout, "".join(seen)
    raise AssertionError("launcher printed no rank pids:\n" + "".join(seen))


def _gone(pids, timeout=20.0):
    import time

    import psutil
    t_end = time.monotonic() + timeout
    while time.monotonic() < t_end:
        alive = []
        for p in pids:
            try:
                if psutil.Process(p).status() != psutil.STATUS_ZOMBIE:
                    alive.append(p)
            except psutil.NoSuchProcess:
                pass
        if not alive:
            return True
        time.sleep(0.1)
    return False


def _kill_all(pids):
    import signal
    for p in pids:
        try:
            os.kill(p, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass


import pytest  # noqa: E402


@pytest.mark.parametrize("fail,stall", [("1", "0"), ("0", "1")])
def test_launcher_failed_rank_stops_the_others(fail, stall):
    """one rank exits non-zero while the other is stuck (as in a collective
    that will never complete): the launcher sees it whatever the failing rank's index, stops
    the stuck rank, returns that failure's status within seconds and leaves no rank alive."""
    import time
    t0 = time.monotonic()
    proc = _launcher({"CODEC_BENCH_FAIL_RANK": fail, "CODEC_BENCH_STALL_RANK": stall})
    pids = []
    try:
        pids, _ = _rank_pids(proc)
        rc = proc.wait(timeout=90)
        err = proc.stderr.read()
        assert rc == 3, err
        assert f"rank {fail} exited with 3" in err
        assert time.monotonic() - t0 < 90
        assert _gone(pids), pids
    finally:
        if proc.poll() is None:
            proc.kill()
        _kill_all(pids)


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGKILL"])
def test_launcher_killed_leaves_no_ranks(sig):
    """A launcher that is terminated (its handler stops the ranks) or killed outright (the
    ranks' parent-death signal) never leaves ranks behind."""
    import signal
    proc = _launcher({"CODEC_BENCH_STALL_RANK": "0", "CODEC_BENCH_FAIL_RANK": "none"})
    pids = []
    try:
        pids, _ = _rank_pids(proc)
        os.kill(proc.pid, getattr(signal, sig))
        rc = proc.wait(timeout=60)
        assert rc != 0
        assert _gone(pids), pids
    finally:
        if proc.poll() is None:
            proc.kill()
        _kill_all(pids)


def test_gpus_world_size_mismatch_is_refused():
    """bench.py --gpus N under a launcher that started a different number of ranks exits
    non-zero before touching the GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_device_uuid_hex():
    """bench._device_uuid: the UUID's bytes as hex; '' when the build exposes none."""
    import types
    import bench
    u = types.SimpleNamespace(bytes=bytes(range(16)))
    assert bench._device_uuid(types.SimpleNamespace(uuid=u)) == bytes(range(16)).hex()
    assert bench._device_uuid(types.SimpleNamespace()) == ""
    assert bench._device_uuid(types.SimpleNamespace(uuid="not-an-object")) == ""
