"""world_size-2 exchange test on the GPU (gloo, both ranks on cuda:0): the real kernels'
records go through the stream-overlapped exchanges the multi-GPU bench uses -- `mark()`
right after the embed, `start()` on the side stream while the extract runs on the launch
stream, `join()` -- with uneven shards (5 slices = 3 + 2).  Every rank recomputes the whole
batch locally and checks that the gathered MED-PEE side information and location-map
prefixes equal it row for row, and the LSB records of its own rows."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _covers(n, h, w, dev, heavy=()):
    """ct12 slices; the slices in `heavy` hold only the values {0, 1, 65534, 65535}, so about
    half their candidates are overflow-prone at any T (their location maps are dense)."""
    from codec_tcc_amd import synth
    out = []
    for i in range(n):
        if i in heavy:
            v = np.random.default_rng(900 + i).integers(0, 4, (h, w))
            out.append(np.where(v < 2, v, 65532 + v).astype(np.uint16))
        else:
            out.append(synth.GENERATORS["ct12"](h, w, 60 + i))
    return torch.from_numpy(np.stack(out)).to(dev)


def _worker(rank, world, port, n, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    ok = True
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import codec_tcc_amd as ct
        from codec_tcc_amd import _lib, framing, synth
        from codec_tcc_amd import distributed as D
        from codec_tcc_amd.pee import PeeCodec
        H = W = 256
        allc = _covers(n, H, W, dev, heavy=(1,))      # slice 1 overflow-heavy: a dense record
        pays = [framing.to_bits(synth.payload(96, 500 + g)) for g in range(n)]
        lo, hi = D.shard_range(n, world, rank)
        B = hi - lo
        # ---- MED-PEE: the whole batch locally (reference rows), then this rank's shard
        full = PeeCodec(n, H, W, dtype="uint16", T=2, device=dev)
        ref = full.embed(allc, pays, check=False)
        codec = PeeCodec(B, H, W, dtype="uint16", T=2, device=dev)
        enc = codec.embed(allc[lo:hi].contiguous(), pays[lo:hi], check=False)
        xch = D.PeeRecordExchange(B, world, dev, n_total=n)
        xch.mark()                                   # records final on the launch stream
        xch.start(enc.meta, enc.lm)                  # side stream ...
        words, cover = codec.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
        gmeta, glm = xch.join()                      # ... joined after the extract was queued
        torch.cuda.synchronize()
        ok &= bool(torch.equal(cover.view(torch.int16), allc[lo:hi].view(torch.int16)))
        ok &= tuple(gmeta.shape) == (n, _lib.PEE_META_BYTES)
        ok &= bool(torch.equal(gmeta, ref.meta))
        recs = ref.records()
        ok &= recs[1].lm_count > 2 * xch.width and recs[0].lm_count <= 2 * xch.width   # dense and sparse rows
        ok &= glm.shape[1] == max((r.end + 64) // 64 for r in recs)
        ok &= bool(torch.equal(glm, D.map_prefix(ref.meta, ref.lm, glm.shape[1])))
        ok &= xch.overflows() == 0
        # ---- LSB records: own rows of the gathered records equal the local packing
        lcodec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
        pl = ct.make_payloads([synth.payload(96, 700 + g) for g in range(lo, hi)], dev)
        lenc = lcodec.encode(allc[lo:hi].contiguous(), pl)
        rx = D.RecordExchange(B, pl.map_words, world, dev, n_total=n)
        rx.mark()
        rx.start(lenc.meta, lenc.maps)
        w2, c2 = lcodec.decode(lenc.stego, lenc.maps, lenc.meta, payload_words=pl.payload_words,
                               map_words=pl.map_words)
        allrec = rx.join()
        torch.cuda.synchronize()
        ok &= bool(torch.equal(c2.view(torch.int16), allc[lo:hi].view(torch.int16)))
        ok &= allrec.shape[0] == n
        mine = D.pack_records(lenc.meta, lenc.maps, out=torch.zeros((B, allrec.shape[1]), dtype=torch.int64,
                                                                      device=dev))
        ok &= bool(torch.equal(rx.own_rows(rank), mine))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, False, repr(e)))
        return
    q.put((rank, bool(ok), ""))


def test_exchanges_on_gpu_streams_world2():
    import torch.multiprocessing as mp
    world, n = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        res = [q.get(timeout=110) for _ in procs]
    finally:
        # a rank that hangs or dies without reporting must not keep holding the GPU for the
        # tests after this one
        for p in procs:
            p.join(timeout=30)
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert len(res) == world and all(ok for _r, ok, _e in res), res
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.timeout(600)
def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2 --backend gloo` with no launcher: the
    script starts two rank processes itself before touching the GPU (both on cuda:0 here),
    and rank 0's JSON line reports the 2-rank job -- the headline MED-PEE step with its
    record exchange, and the C4 leg (256 x 512^2 per rank, T = auto, exchange)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--backend", "gloo", "--batch", "8",
           "--size", "512", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--c2", "0", "--no-profile",
           "--payload-chars", "256"]   # within a 512^2 slice's T = 2 capacity
    r = subprocess.run(cmd, env=env, cwd=repo, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 16
    assert out["roundtrip_ok"] is True and out["pee"]["exchange_ok"] is True, out["pee"]
    assert out["pee"]["distributed"]["narrow_gathers"] == 0
    assert out["lsb"]["roundtrip_ok"] is True and out["lsb"]["exchange_ok"] is True, out["lsb"]
    assert out["c4"]["roundtrip_ok"] is True and out["c4"]["exchange_ok"] is True, out["c4"]
    # the per-rank records: one per rank, in rank order, over the named backend
    rk = out["ranks"]
    assert [r["rank"] for r in rk] == [0, 1] and all(r["world_size"] == 2 and r["backend"] == "gloo" for r in rk)
    assert all(r["ms_per_step"] > 0 and r["kernels_only_ms"] > 0 and r["pci"] for r in rk), rk
    assert out["distinct_devices"] == 1          # both gloo ranks share the box's one GPU
    assert not any(k.startswith("_") for k in out["pee"]), out["pee"].keys()
    # a launcher that started a different number of ranks is refused
    bad = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2"],
                         env=dict(env, WORLD_SIZE="1", RANK="0"), cwd=repo, capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr


@pytest.mark.timeout(900)
def test_bench_eight_ranks_rehearsal():
    """the driver's 8-GPU run rehearsed at 8 ranks on the box's one GPU
    (gloo): `bench.py --gpus 8` starts 8 fresh rank processes before any GPU call, every
    exchange (headline MED-PEE, LSB, the C4 leg's 256 x 512^2 per rank) round-trips exactly
    with no narrow gather, the `ranks` array names all 8 ranks, and no rank pid survives."""
    import json
    import subprocess
    import sys
    import threading

    from test_bench_host import _gone, _kill_all
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "-u", os.path.join(repo, "bench.py"), "--gpus", "8", "--backend", "gloo", "--batch", "4",
           "--size", "512", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--c2", "0", "--no-profile",
           "--payload-chars", "256"]
    proc = subprocess.Popen(cmd, env=env, cwd=repo, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    pids, err = [], []

    def drain():                 # keep the launcher's stderr moving; pick up the rank pids
        for line in proc.stderr:
            err.append(line)
            if line.startswith("bench.py: rank pids "):
                pids.extend(int(x) for x in line.split()[3:])
    t = threading.Thread(target=drain, daemon=True)
    t.start()
    try:
        out_s = proc.stdout.read()
        rc = proc.wait(timeout=840)
        t.join(timeout=10)
        assert rc == 0, "".join(err)[-4000:]
        assert len(pids) == 8, pids
        lines = [ln for ln in out_s.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, out_s[-2000:]
        out = json.loads(lines[0])
        assert out["n_gpus"] == 8 and out["config"]["global_batch"] == 32
        assert out["roundtrip_ok"] is True and out["pee"]["exchange_ok"] is True, out["pee"]
        assert out["pee"]["distributed"]["narrow_gathers"] == 0
        assert out["lsb"]["roundtrip_ok"] is True and out["lsb"]["exchange_ok"] is True, out["lsb"]
        assert out["c4"]["roundtrip_ok"] is True and out["c4"]["exchange_ok"] is True, out["c4"]
        assert out["c4"]["distributed"]["narrow_gathers"] == 0
        rk = out["ranks"]
        assert [r["rank"] for r in rk] == list(range(8)), rk
        assert all(r["world_size"] == 8 and r["backend"] == "gloo" and r["ms_per_step"] > 0 for r in rk), rk
        assert len({r["pid"] for r in rk}) == 8 and {r["pid"] for r in rk} == set(pids)
        assert _gone(pids), pids
    finally:
        if proc.poll() is None:
            proc.kill()
        _kill_all(pids)


@pytest.mark.timeout(200)
def test_bench_failed_rank_on_gpu_box():
    """VERDICT r3 item 1 on the GPU box: `bench.py --gpus 2 --backend gloo` with rank 1 made to
    exit right after init_process_group while rank 0 is stuck returns that status within a
    minute and leaves no rank alive (the CPU suite runs the same cases, test_bench_host.py)."""
    import time

    from test_bench_host import _gone, _kill_all, _launcher, _rank_pids
    t0 = time.monotonic()
    proc = _launcher({"CODEC_BENCH_FAIL_RANK": "1", "CODEC_BENCH_STALL_RANK": "0"})
    pids = []
    try:
        pids, _ = _rank_pids(proc)
        rc = proc.wait(timeout=120)
        err = proc.stderr.read()
        assert rc == 3 and "rank 1 exited with 3" in err, err
        assert time.monotonic() - t0 < 90
        assert _gone(pids), pids
    finally:
        if proc.poll() is None:
            proc.kill()
        _kill_all(pids)


def _rccl_worker(port, q):
    """One rank over the nccl (= RCCL) backend: the exchanges' RCCL branches
    (all_gather_into_tensor, all_reduce) on real kernel records."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl"
        import codec_tcc_amd as ct
        from codec_tcc_amd import framing, synth
        from codec_tcc_amd import distributed as D
        from codec_tcc_amd.pee import PeeCodec
        n, H, W = 3, 256, 256
        allc = _covers(n, H, W, dev)
        codec = PeeCodec(n, H, W, dtype="uint16", T=2, device=dev)
        enc = codec.embed(allc, [framing.to_bits(synth.payload(96, 40 + g)) for g in range(n)])
        xch = D.PeeRecordExchange(n, 1, dev)
        ok = True
        for _ in range(3):                      # first call agrees the width; later ones carry it
            xch.mark()
            xch.start(enc.meta, enc.lm)
            gmeta, glm = xch.join()
            torch.cuda.synchronize()
            ok &= bool(torch.equal(gmeta, enc.meta))
            ok &= bool(torch.equal(glm, D.map_prefix(enc.meta, enc.lm, glm.shape[1])))
        ok &= xch.overflows() == 0 and D.agree_max(7, device=dev) == 7
        # a later step whose maps need a wider record (an overflow-heavy slice
        # appears): join() -- no explicit verify() -- still returns every map exactly
        w0 = xch.width
        hc = _covers(n, H, W, dev, heavy=(2,))
        enc2 = codec.embed(hc, [framing.to_bits(synth.payload(96, 40 + g)) for g in range(n)], check=False)
        xch.mark()
        xch.start(enc2.meta, enc2.lm)
        gmeta, glm = xch.join()
        torch.cuda.synchronize()
        ok &= xch.width > w0 and xch.overflows() == 0
        ok &= bool(torch.equal(gmeta, enc2.meta))
        ok &= bool(torch.equal(glm, D.map_prefix(enc2.meta, enc2.lm, glm.shape[1])))
        lcodec = ct.Codec(n, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
        pl = ct.make_payloads([synth.payload(96, 70 + g) for g in range(n)], dev)
        lenc = lcodec.encode(allc, pl)
        rx = D.RecordExchange(n, pl.map_words, 1, dev)
        rx.mark()
        rx.start(lenc.meta, lenc.maps)
        allrec = rx.join()
        torch.cuda.synchronize()
        ok &= bool(torch.equal(allrec, D.pack_records(lenc.meta, lenc.maps)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((False, repr(e)))
        return
    q.put((bool(ok), ""))


def test_exchanges_over_rccl_world1():
    """The RCCL code path of the record exchanges (the 8-GPU bench's collectives) with one
    rank on the box's one GPU: RCCL refuses two ranks on one device, so this is the only RCCL
    run possible here; the multi-rank path is covered over gloo above."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        ok, err = q.get(timeout=110)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
            p.join(timeout=10)
    assert ok, err


def test_pee_record_kernels_match_host_rule():
    """codec_pee_pack_records / codec_pee_unpack_records on real embed outputs (ct12 slices
    with near-empty maps, one overflow-heavy slice) equal the host restatement of the record
    rule (distributed.pack_pee_records on CPU tensors) word for word, and unpacking returns
    every map exactly whenever the width is the needed one or wider."""
    from codec_tcc_amd import distributed as D
    from codec_tcc_amd import framing, synth
    from codec_tcc_amd.pee import PeeCodec
    dev = torch.device("cuda", 0)
    n, H, W = 5, 256, 256
    covers = _covers(n, H, W, dev, heavy=(3,))
    codec = PeeCodec(n, H, W, dtype="uint16", T=2, device=dev)
    enc = codec.embed(covers, [framing.to_bits(synth.payload(64 + 40 * g, 10 + g)) for g in range(n)], check=False)
    lm_cpu, meta_cpu = enc.lm.cpu(), enc.meta.cpu()
    need = int(D.record_width_needed(enc.meta, codec.lm_words))
    assert need == int(D.record_width_needed(meta_cpu, codec.lm_words)) > 1
    cols = int(D.dense_words_needed(enc.meta))
    want = D.map_prefix(meta_cpu, lm_cpu, cols)
    for width in (1, need, need + 3):
        rec = D.pack_pee_records(enc.meta, enc.lm, width)
        torch.cuda.synchronize()
        assert torch.equal(rec.cpu(), D.pack_pee_records(meta_cpu, lm_cpu, width)), width
        meta2, lm2 = D.unpack_pee_records(rec, cols)
        assert torch.equal(meta2.cpu(), meta_cpu)
        _m, lm2_cpu = D.unpack_pee_records(rec.cpu(), cols)
        assert torch.equal(lm2.cpu(), lm2_cpu), width
        if width >= need:
            assert torch.equal(lm2.cpu(), want), width
        else:
            assert not torch.equal(lm2.cpu(), want)      # the heavy slice is cut: what overflows() flags
