#!/usr/bin/env python3
"""Benchmark of the MED-PEE embed+extract hot path (BASELINE.json's metric) on MI355X.

One step = codec_pee_embed (cover -> stego: MED prediction, error expansion / shifting,
location map, per-slice side information) + codec_pee_extract (stego -> exact payload +
restored cover) over one batch of synthetic uint16 slices already resident in HBM, plus
(N > 1) the RCCL all-gather of every slice's side information and location map (on a side
stream after embed, overlapped with extract).  `value` / `ms_per_step` are that step.

Side legs in the same JSON line: `lsb` (the reference's own bit-plane LSB pixel path,
src/codec.py:412-487 + 752-793, bit-exact with it), `inplace` (the PEE step with stego =
cover), `quality` / `pee.quality` (src/mse.py metrics of the LSB and the MED-PEE stego),
`c3` (256 x 512^2), `c2` (1 x 2048^2); at N > 1 `ranks` (what each rank ran on).  Prints ONE
JSON line (rank 0).

    python bench.py                              # N=1, 256 x 2048^2 ct12, K=20, W=3
    torchrun --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mpixels/s PEE embed+extract, 2048² uint16 batch; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="slices per GPU")
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--kind", default="ct12", choices=["ct12", "u16"])
    ap.add_argument("--payload-chars", type=int, default=1024)
    ap.add_argument("--pee-T", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU-baseline budget of the MED-PEE oracle (0 = skip every CPU baseline)")
    ap.add_argument("--cpu-ref-seconds", type=float, default=6.0,
                    help="CPU-baseline budget of the reference-path (LSB) oracle")
    ap.add_argument("--cpu-pool", type=int, default=16,
                    help="workers of the pooled CPU baselines (the box's CPU share per GPU is 16; 0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event passes")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    ap.add_argument("--lsb", type=int, default=1, help="also time the reference's LSB bit-plane path")
    ap.add_argument("--c3", type=int, default=1, help="also time BASELINE config C3 (256 x 512^2)")
    ap.add_argument("--c2", type=int, default=1, help="also time BASELINE config C2 (1 x 2048^2, latency)")
    ap.add_argument("--c2-graph", type=int, default=0,
                    help="C2 MED-PEE leg replayed from a HIP graph (the eager time is reported too); off by "
                         "default: measured slower, 0.0307 vs 0.0242 ms per step")
    return ap.parse_args()


def make_covers(torch, kind, b, h, w, device, seed):
    """Synthetic slices generated on the device (no host->device GBs)."""
    if kind == "u16":
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        x = torch.randint(0, 65536, (b, h, w), generator=g, device=device, dtype=torch.int32)
        return x.to(torch.uint16)
    ys = torch.arange(h, device=device, dtype=torch.float32).view(1, h, 1)
    xs = torch.arange(w, device=device, dtype=torch.float32).view(1, 1, w)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((b, h, w), dtype=torch.uint16, device=device)
    for i in range(b):
        base = (torch.sin(xs / 97.0 + (seed + i)) + torch.cos(ys / 61.0) + 2.0) / 4.0 * 4095.0 * 0.8
        noise = torch.randn((1, h, w), generator=g, device=device) * 16.0
        out[i] = torch.clamp(torch.round(base + noise), 0, 4095).to(torch.int32).to(torch.uint16)[0]
    return out


def pmc_traffic(kernel: str, b: int, h: int, w: int, kind: str, targs=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_summary.py: FETCH_SIZE x2 (gfx950 correction)
    + WRITE_SIZE, KB -> bytes), when it was collected on this exact configuration.

    The summaries are keyed per template instantiation (`k<unsigned short, true, ...>`):
    `kernel` is the bare name, and `targs` {index: "value"} selects among its
    instantiations by template argument (e.g. {2: "true"} = the in-place PEE kernels);
    the lookup succeeds only when exactly one instantiation matches."""
    d = None
    for name in ("pmc_traffic.json", "pmc_traffic_c3.json", "pmc_traffic_c2.json"):   # headline, C3, C2 shapes
        path = os.path.join(REPO, "profiles", name)
        try:
            with open(path) as f:
                cand = json.load(f)
        except (OSError, ValueError):
            continue
        cfg = cand.get("config", {})
        if (cfg.get("batch"), cfg.get("h"), cfg.get("w"), cfg.get("kind")) == (b, h, w, kind):
            d = cand
            break
    if d is None:
        return None
    hits = []
    for n, v in d.get("kernels", {}).items():
        bare, _, rest = n.partition("<")
        if bare != kernel:
            continue
        args = [a.strip() for a in rest.rstrip(">").split(",")] if rest else []
        if all(i < len(args) and args[i] == val for i, val in (targs or {}).items()):
            hits.append((n, v))
    if len(hits) != 1:
        return None
    name, k = hits[0]
    return {"hbm_bytes_per_launch": k["hbm_bytes_per_launch"], "source": d.get("source", path), "instance": name}


def _cpu_model() -> str:
    """The host CPU (report the model beside the core count)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------------ CPU baselines
_CPU_IMGS = {}
CPU_DISTINCT = 8


def _cpu_img(size, kind, seed):
    """Synthetic cover for the CPU baselines: CPU_DISTINCT distinct slices, generated once
    (generating a 2048^2 ct12 slice costs ~3x the oracle's PEE embed + extract of it)."""
    from codec_tcc_amd import synth
    key = (size, kind, seed % CPU_DISTINCT)
    if key not in _CPU_IMGS:
        _CPU_IMGS[key] = synth.GENERATORS[kind](size, size, 1000 + seed % CPU_DISTINCT)
    return _CPU_IMGS[key]


def _pee_cpu_slice(size, kind, chars, T, seed):
    """One oracle MED-PEE embed + extract of a slice (own payload): (pixels, seconds)."""
    from codec_tcc_amd import framing, synth
    from oracle import pee_cpu as P
    img = _cpu_img(size, kind, seed)
    bits = framing.to_bits(synth.payload(chars, 99 + seed))
    t0 = time.perf_counter()
    st, side = P.pee_embed(img, bits, T, truncate=True)
    P.pee_extract(st, side)
    return img.size, time.perf_counter() - t0


def _lsb_cpu_slice(size, kind, chars, seed):
    """One oracle encode+decode of the reference's LSB path (decomposition + hybrid embed +
    merge + extract_local_planes + decode_message): (pixels, seconds)."""
    from codec_tcc_amd import synth
    from oracle import ref_cpu as R
    img = _cpu_img(size, kind, seed)
    bits = R.message_to_bits(synth.payload(chars, 7 + seed))
    t0 = time.perf_counter()
    enc = R.encode_slice(img, bits, beta=0.4, sb=16)
    R.decode_slice(enc["stego"], enc["bitmaps"], enc["s"], enc["segments_lengths"], enc["segment_indices"])
    return img.size, time.perf_counter() - t0


def _timed_loop(fn, budget_s):
    """Run fn on successive slices until budget_s seconds of timed oracle work."""
    px = n = 0
    t_work = 0.0
    while n == 0 or t_work < budget_s:
        p, t = fn(1000 + n)
        px += p
        t_work += t
        n += 1
    return px, n, t_work


def _cgroup_cpu_quota():
    """CPU quota of this process's cgroup in cores (cgroup v2 cpu.max / v1 cfs files), or None
    when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = float(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def _affinity():
    """Host cores this process may run on (sorted)."""
    try:
        return sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):   # pragma: no cover - non-Linux
        return list(range(os.cpu_count() or 1))


_PIN_NEXT = None


def _pin_worker(cores):
    """Pool initializer: pin this worker to the next core of `cores` (one core each)."""
    with _PIN_NEXT.get_lock():
        i = _PIN_NEXT.value
        _PIN_NEXT.value += 1
    os.sched_setaffinity(0, {cores[i % len(cores)]})


def _pinned_pool(workers, cores):
    """A fork pool of `workers` processes, worker i pinned to cores[i]."""
    import multiprocessing as mp
    global _PIN_NEXT
    ctx = mp.get_context("fork")
    _PIN_NEXT = ctx.Value("i", 0)
    return ctx.Pool(workers, initializer=_pin_worker, initargs=(list(cores),))


def _cpu_baseline_work(args):
    size, kind, chars = args.size, args.kind, args.payload_chars
    px, n, t = _timed_loop(lambda s: _pee_cpu_slice(size, kind, chars, args.pee_T, s), args.cpu_seconds)
    out = {"value": round(px / t / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
           "sample": f"{n} x {size}x{size} {kind} uint16 slice runs ({CPU_DISTINCT} distinct covers, "
                     f"distinct {chars}-char payloads), T={args.pee_T}: oracle/pee_cpu.py embed + extract "
                     f"(numpy), 1 process pinned to one core; seconds = timed oracle work",
           "seconds": round(t, 2), "cpu_model": _cpu_model()}
    if args.cpu_ref_seconds > 0:
        px, n, t = _timed_loop(lambda s: _lsb_cpu_slice(size, kind, chars, s), args.cpu_ref_seconds)
        out["reference_path"] = {
            "value": round(px / t / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"{n} x {size}x{size} {kind} slice runs ({CPU_DISTINCT} distinct covers): the reference's "
                      f"numpy loop (oracle/ref_cpu.py: decompose + hybrid embed + merge + "
                      f"extract_local_planes + decode_message), 1 process pinned to one core",
            "seconds": round(t, 2)}
    return out


def cpu_baseline(args):
    """The MED-PEE oracle (oracle/pee_cpu.py, vectorised numpy) on this host, ONE process
    pinned to one core (SURVEY §8(d) / BASELINE.md: `taskset -c 0`; here a forked child with
    sched_setaffinity to the first core this process may use), on distinct synthetic slices
    of the benchmark's shape until the budget is used; beside it the reference-path oracle
    (numpy restatement of src/codec.py, bit-identical to it).  Call before the GPU is
    initialised (the child is forked)."""
    cores = _affinity()
    with _pinned_pool(1, cores[:1]) as pool:
        out = pool.apply(_cpu_baseline_work, (args,))
    out["pinned_core"] = cores[0]
    out["cores_available"] = len(cores)
    return out


def _pool_job(job):
    which, size, kind, chars, T, seed = job
    return _pee_cpu_slice(size, kind, chars, T, seed) if which == "pee" else _lsb_cpu_slice(size, kind, chars, seed)


def cpu_baseline_pool(args, which: str, per_worker: int = 0):
    """The same oracle work over a process pool (one worker per host core),
    each worker pinned to its own core.  The pool has min(len(sched_getaffinity), cgroup CPU
    quota, --cpu-pool) workers: on the GPU box the affinity set is the whole machine (256
    cores) while the pool's rules give one GPU's job a 16-core share (--cpu-pool 16), so a
    whole-machine pool would time-slice 256 workers on that share.  The whole-host figure is
    therefore reported beside it as an extrapolation (`host_extrapolated`: the pool's per-core
    rate x the cores in the affinity set), labelled as such.  Forked BEFORE the GPU is
    initialised in this process; the covers are generated in the parent first, so the wall
    clock holds the fork and the oracle work."""
    cores = _affinity()
    quota = _cgroup_cpu_quota()
    usable = len(cores) if quota is None else max(1, min(len(cores), int(quota)))
    workers = max(1, min(usable, int(args.cpu_pool)))
    per_worker = per_worker or (40 if which == "pee" else 4)   # ~2 s of oracle work per worker
    for i in range(CPU_DISTINCT):
        _cpu_img(args.size, args.kind, i)
    jobs = [(which, args.size, args.kind, args.payload_chars, args.pee_T, 2000 + i) for i in range(workers * per_worker)]
    t0 = time.perf_counter()
    with _pinned_pool(workers, cores[:workers]) as pool:
        res = pool.map(_pool_job, jobs, chunksize=1)
    wall = time.perf_counter() - t0
    px = sum(r[0] for r in res)
    rate = px / wall / 1e6
    return {"value": round(rate, 3), "unit": "Mpixels/s", "cores": workers, "kind": "port",
            "sample": f"{len(jobs)} x {args.size}x{args.size} {args.kind} slices ({which} oracle) over a "
                      f"{workers}-process pool, one core per worker (fork; {CPU_DISTINCT} distinct covers "
                      f"generated beforehand), wall clock",
            "seconds": round(wall, 2), "cpu_model": _cpu_model(), "cores_available": len(cores),
            "cgroup_cpu_quota": quota, "per_gpu_share_cores": int(args.cpu_pool),
            "pinned_cores": cores[:workers],
            # NOT a measurement: the pool's per-core rate scaled to every core of the affinity
            # set (the oracle slices are independent, one per core: linear up to memory bandwidth)
            "host_extrapolated": {"value": round(rate / workers * len(cores), 1), "cores": len(cores),
                                  "basis": "pool per-core rate x cores_available (extrapolated, not run)"}}


# ------------------------------------------------------------------ helpers
def _profile(lib, _lib, fn, steps):
    import ctypes as C
    import torch
    cap = 64 * steps
    _lib.check(lib.codec_profile_begin(cap), "codec_profile_begin")
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    ms = (C.c_float * cap)()
    tags = (C.c_int32 * cap)()
    n = lib.codec_profile_end(ms, tags, cap)
    out = {}
    for i in range(max(n, 0)):
        out.setdefault(_lib.KERNEL_TAGS.get(tags[i], str(tags[i])), []).append(ms[i])
    return {k: float(np.mean(v)) for k, v in out.items()}


def _timed(torch, dist, world, dev, fn, steps, local=None):
    """Barrier + synchronize on both sides of exactly `steps` calls; max over ranks (s).
    `local` (a dict) receives this rank's own figure under "s" (the per-rank record)."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if local is not None:   # this rank's own work, before the closing barrier waits for the others
        local["s"] = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def payload_equal(got_words, want_words, nbits) -> bool:
    """Recovered payload words == embedded ones on each slice's first nbits[b] bits, and
    no bit set past them (LSB-first packing, framing.pack_bits)."""
    g = got_words.detach().cpu().numpy().view(np.uint64)
    w = want_words.detach().cpu().numpy().view(np.uint64)
    nw = min(g.shape[1], w.shape[1])
    idx = np.arange(g.shape[1] * 64).reshape(g.shape[1], 64)
    for b, n in enumerate(nbits):
        mask = np.packbits(idx < int(n), axis=None, bitorder="little").view(np.uint64)
        if np.any((g[b] & mask)[:nw] != (w[b] & mask)[:nw]) or np.any(g[b] & ~mask):
            return False
    return True


def _roof(kernel, by, t_ms, traffic=None):
    ach = by / (t_ms / 1e3) / 1e9
    r = {"bound": "hbm", "kernel": kernel, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "algorithmic_bytes_per_launch": int(by),
         "avg_launch_ms": round(t_ms, 4)}
    if traffic is not None:
        r["traffic"] = traffic["hbm_bytes_per_launch"]
        r["traffic_source"] = traffic["source"]
        r["traffic_instance"] = traffic.get("instance")
    return r


# ------------------------------------------------------------------ MED-PEE (headline)
def bench_pee(args, torch, dist, world, rank, dev, covers, B, H, W, *, inplace=False, exchange=False,
              steps=None, kind=None, T=None, graph=False):
    """MED-PEE embed + extract over one resident batch (1 KB payload per slice).
    Out of place at 2048^2: k_pee_embed1 (one pass: copy + look-back cursor + embed) and
    k_pee_extract1 (one pass: copy + look-back cursor + recover).  In place (and small
    slices, e.g. C3) at chip-filling batch sizes: the slice-serial k_pee_embed_ss /
    k_pee_extract_ss (one workgroup per slice); in place only the items up to each slice's
    `end` are read and written.  exchange (N > 1):
    the side information + location maps of every slice to every rank
    (distributed.PeeRecordExchange), on a side stream overlapped with extract."""
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd import distributed as D
    from codec_tcc_amd.pee import PeeCodec, PeeEncoded
    steps = args.steps if steps is None else steps
    kind = args.kind if kind is None else kind
    T = args.pee_T if T is None else T
    codec = PeeCodec(B, H, W, dtype="uint16", T=T, device=dev)
    pay = [synth.payload(args.payload_chars, 99 + rank * B + i) for i in range(B)]
    packed = codec.pack_payloads(pay)
    work = covers.clone() if inplace else None
    stego = work if inplace else torch.empty_like(covers)
    cov2 = work if inplace else torch.empty_like(covers)
    src = work if inplace else covers
    lm = torch.empty((B, codec.lm_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=dev)
    pw = packed[0].shape[1]
    outw = torch.empty((B, pw), dtype=torch.int64, device=dev)
    xch = D.PeeRecordExchange(B, world, dev) if exchange else None

    def kernels():
        codec.embed(src, None, stego=stego, lm=lm, meta=meta, packed=packed, check=False)
        if xch is not None:
            xch.mark()
        codec.extract(stego, meta, lm, payload_words=pw, cover=cov2, payload=outw)

    def step():
        kernels()
        if xch is not None:
            xch.start(meta, lm)
            xch.join_records()     # no host read in the timed step; overflows() checked after

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if graph:
        # launch-bound shapes (C2): the same four launches replayed from one HIP graph
        # (codec_tcc_amd/graphs.py); the eager loop's time is reported beside it
        from codec_tcc_amd import graphs
        el_eager = _timed(torch, dist, world, dev, step, steps)
        g = graphs.capture(kernels)
        outw.zero_()
        cov2.zero_()
        step = g.replay
        for _ in range(args.warmup):
            step()
    mine = {}
    el = _timed(torch, dist, world, dev, step, steps, local=mine)
    # correctness of the state the timed steps left (outside the timed region): restored
    # cover, recovered payload bits, per-slice status and the decode-side look-back flag
    recs = PeeEncoded(stego, lm, meta, packed[1], pw).records()
    nbits = [r.L if r.status == 0 else r.capacity for r in recs]
    cover_ok = bool(torch.equal(cov2.view(torch.int16), covers.view(torch.int16)))
    pay_ok = payload_equal(outw, packed[0], nbits)
    flags_ok = all(r.status in (0, 1) for r in recs) and not codec.lookback_failed(pw)
    res = {"value": round(B * H * W * world * steps / el / 1e6, 1), "unit": "Mpixels/s",
           "ms_per_step": round(el / steps * 1e3, 4), "T": T,
           "_rank_ms_per_step": round(mine["s"] / steps * 1e3, 4),
           "roundtrip_ok": cover_ok and pay_ok and flags_ok and all(r.status == 0 for r in recs),
           "cover_ok": cover_ok, "payload_ok": pay_ok, "lookback_ok": flags_ok,
           "end_candidates_mean": float(np.mean([r.end + 1 for r in recs])),
           # the scheme's capacity bound: only the (odd, odd) lattice -- a quarter of the
           # pixels -- can carry bits (the rest is the untouched MED context)
           "candidates_per_slice": (H // 2) * (W // 2),
           # slices whose payload exceeds the T-capacity (truncated, still exactly reversible;
           # roundtrip_ok then reads False): uniform-noise slices at T=2
           "overflow_slices": int(sum(1 for r in recs if r.status == 1)),
           "repaired_slices": codec.repaired(pw)}
    if graph:
        res["launch"] = "hip_graph"
        res["eager"] = {"value": round(B * H * W * world * steps / el_eager / 1e6, 1),
                        "ms_per_step": round(el_eager / steps * 1e3, 4)}
    if T == "auto":
        res["T_chosen"] = {str(t): int(sum(1 for r in recs if r.T == t)) for t in sorted({r.T for r in recs})}
    if xch is not None:
        # every timed gather was wide enough (device-side count, read once now), this rank's
        # rows of the last one are its own records, and they decode to its own metas and maps
        narrow = xch.overflows()
        own = xch.own_rows(rank)
        om, ol = D.unpack_pee_records(own, int(D.dense_words_needed(meta)))
        res["exchange_ok"] = narrow == 0 and \
            bool(torch.equal(own, D.pack_pee_records(meta, lm, xch.width))) and \
            bool(torch.equal(om, meta)) and bool(torch.equal(ol, D.map_prefix(meta, lm, ol.shape[1])))
        t_g = _timed(torch, dist, world, dev, lambda: (xch.start(meta, lm), xch.join_records()), steps) / steps
        mine_k = {}
        t_k = _timed(torch, dist, world, dev, kernels, steps, local=mine_k) / steps
        res["_rank_kernels_only_ms"] = round(mine_k["s"] / steps * 1e3, 4)
        res["distributed"] = {
            "allgather_ms": round(t_g * 1e3, 4),
            "allgather_bytes": xch.gathered_bytes,
            "record_bytes_per_slice": xch.record_bytes,
            "dense_prefix_bytes_per_slice": 64 + 8 * int(D.dense_words_needed(meta)),
            "collectives_per_step": 1,
            "narrow_gathers": narrow,
            "record_map_words": xch.width,
            "kernels_only_ms_per_step": round(t_k * 1e3, 4),
            "kernels_only_value": round(B * H * W * world / t_k / 1e6, 1)}
    kern = _profile(_lib.load(), _lib, kernels, steps) if not args.no_profile else {}
    res["kernels_ms"] = {k: round(v, 4) for k, v in kern.items()}
    # the launch path the dispatcher chose (codec_pee.hip pee_use_slice_serial): the
    # slice-serial kernels for chip-filling batches in place / small slices, else look-back
    emb = next((k for k in ("k_pee_embed_res", "k_pee_embed_ss_auto", "k_pee_embed_ss", "k_pee_embed1", "k_pee_scan")
                if k in kern), None)
    ext = next((k for k in ("k_pee_extract_ss", "k_pee_extract1") if k in kern), None)
    res["embed_kernel"], res["extract_kernel"] = emb, ext
    # PMC instantiation of each tag: template argument 2 is INPLACE for every PEE kernel; the
    # slice-serial embed's argument 5 is AUTO (the capacity phase fused in, codec_pee_embed_auto)
    ip = "true" if inplace else "false"
    targs = {"k_pee_embed_ss": ("k_pee_embed_ss", {2: ip, 5: "false"}),
             "k_pee_embed_ss_auto": ("k_pee_embed_ss", {2: ip, 5: "true"}),
             "k_pee_extract_ss": ("k_pee_extract_ss", {2: ip}),
             "k_pee_embed1": ("k_pee_embed1", {2: ip}),
             "k_pee_extract1": ("k_pee_extract1", {2: ip})}

    def traffic(tag):
        name, ta = targs.get(tag, (tag, None))
        return pmc_traffic(name, B, H, W, kind, ta)

    if not inplace:
        res["_stego"] = stego      # the headline's stego quality (bench_quality, outside the timings)
    if inplace:
        # algorithmic bytes: every 8-px x 2-row item up to the one holding `end` is read
        # (candidates + their neighbours), its candidate row written back
        prefix_px = sum(((r.end // 4) + 1) * 16 for r in recs if r.end >= 0)
        by = prefix_px * 2 + prefix_px // 2 * 2
        # only the prefix is processed in place: `value` counts those pixels; the whole
        # slices' pixel rate (what the out-of-place step processes) is `nominal_mpx_s`
        res["nominal_mpx_s"] = res["value"]
        res["value"] = round(prefix_px * world * steps / el / 1e6, 1)
        res["value_basis"] = ("pixels read up to each slice's `end` (items of 8 px x 2 rows); nominal_mpx_s "
                              "counts every pixel of the batch")
        res["touched_fraction"] = round(prefix_px / (B * H * W), 4)
        res["prefix_pixels_per_step"] = int(prefix_px)
        if emb in ("k_pee_embed_res", "k_pee_embed_ss_auto", "k_pee_embed_ss", "k_pee_embed1") and kern[emb] > 0:
            res["roofline"] = _roof(emb, by, kern[emb], traffic(emb))
        if ext and kern[ext] > 0:
            # extract reads the same items plus their location-map words, writes the rows back
            res["extract_roofline"] = _roof(ext, by, kern[ext], traffic(ext))
        return res
    if emb:
        res["roofline"] = _roof(emb, B * H * W * 4, kern[emb], traffic(emb))   # read cover + write stego
    if ext:
        res["extract_roofline"] = _roof(ext, B * H * W * 4, kern[ext], traffic(ext))
    t_emb = sum(kern.get(k, 0.0) for k in ("k_pee_embed_res", "k_pee_embed_ss_auto", "k_pee_embed_ss", "k_pee_embed1",
                                           "k_pee_scan", "k_pee_locate", "k_pee_embed")) / 1e3
    if t_emb > 0:
        # north-star figure: cover bytes read / t_embed / peak (an out-of-place embed also
        # writes as many bytes, so this cannot exceed ~0.5 of the shared HBM bandwidth)
        res["embed_read_roofline_frac"] = round(B * H * W * 2 / t_emb / 1e9 / HBM_PEAK_GBS, 4)
    return res


# ------------------------------------------------------------------ LSB (reference path)
def bench_lsb(args, torch, dist, world, rank, dev, covers, B, H, W, *, exchange=False, steps=None, kind=None,
              seed0=7):
    """The reference's bit-plane LSB path: encode (codec_plan: histogram/decision/block-search
    scan + stego copy, fused embed) + decode (codec_extract: cover restore stream + payload
    gather); N > 1 adds the RCCL all-gather of the slice records + packed maps."""
    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd import distributed as D
    steps = args.steps if steps is None else steps
    kind = args.kind if kind is None else kind
    codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
    pl = ct.make_payloads([synth.payload(args.payload_chars, seed0 + rank * B + i) for i in range(B)], dev)
    stego = torch.empty((B, H, W), dtype=torch.uint16, device=dev)
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    cover_out = torch.empty((B, H, W), dtype=torch.uint16, device=dev)
    payload_out = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)
    xch = D.RecordExchange(B, pl.map_words, world, dev) if exchange else None

    def kernels():
        codec.encode(covers, pl, stego=stego, maps=maps, meta=meta, check=False)
        if xch is not None:
            xch.mark()
        codec.decode(stego, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words,
                     cover=cover_out, payload=payload_out)

    def step():
        kernels()
        if xch is not None:
            xch.start(meta, maps)
            xch.join()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    el = _timed(torch, dist, world, dev, step, steps)
    recs = ct.meta_records(meta)
    cover_ok = bool(torch.equal(cover_out.view(torch.int16), covers.view(torch.int16)))
    pay_ok = payload_equal(payload_out, pl.words, [r.total_used for r in recs]) and \
        all(r.total_used == n for r, n in zip(recs, pl.lengths))
    # a non-zero status (e.g. 2 = a split decision timed out) means s may differ from the
    # reference's decision even though the round trip itself is exact
    status_ok = all(r.status == 0 for r in recs)
    res = {"value": round(B * H * W * world * steps / el / 1e6, 1), "unit": "Mpixels/s",
           "ms_per_step": round(el / steps * 1e3, 4), "roundtrip_ok": cover_ok and pay_ok and status_ok,
           "cover_ok": cover_ok, "payload_ok": pay_ok, "status_ok": status_ok, "s_values": sorted({r.s for r in recs}),
           # the guard-banded s decision: slices settled from H(X) vs those inside the 1e-9 band
           # (decided by the numpy-order joint sums)
           "decide": {"guarded": sum(1 for r in recs if r.flags & _lib.FLAG_INFO_FAST),
                      "guard_fallbacks": sum(1 for r in recs if r.flags & _lib.FLAG_GUARD_FALLBACK)},
           "path": "the reference's pixel path (bit-plane LSB embed + true decode, src/codec.py:412-487, "
                   "752-793), bit-exact with it"}
    if xch is not None:   # this rank's rows of the gathered records are its own packed records
        res["exchange_ok"] = bool(torch.equal(xch.own_rows(rank), D.pack_records(meta, maps, out=torch.zeros_like(xch.record)[:B])))
        t_g = _timed(torch, dist, world, dev, lambda: (xch.start(meta, maps), xch.join()), steps) / steps
        t_k = _timed(torch, dist, world, dev, kernels, steps) / steps
        res["distributed"] = {"allgather_ms": round(t_g * 1e3, 4),
                              "allgather_bytes": int(xch.padded.numel() * 8),
                              "kernels_only_ms_per_step": round(t_k * 1e3, 4),
                              "kernels_only_value": round(B * H * W * world / t_k / 1e6, 1)}
    kern = _profile(_lib.load(), _lib, kernels, steps) if not args.no_profile else {}
    res["kernels_ms"] = {k: round(v, 4) for k, v in kern.items()}
    # the copying scan (fused with the decision and embed at C3-like shapes: k_scan_decide)
    sk = next((k for k in ("k_scan_rows", "k_scan_fast", "k_scan_decide") if k in kern), None)
    if sk:   # read cover + write stego (uint16)
        res["roofline"] = _roof(sk, B * H * W * 4, kern[sk], pmc_traffic(sk, B, H, W, kind))
    res["_stego"] = stego
    return res


def bench_lsb_inplace(args, torch, dist, world, dev, covers, B, H, W):
    """The reference-algorithm step in place: codec_plan only reads the cover (no stego copy),
    codec_embed rewrites the <= payload-size window pixels of the same buffer, codec_extract
    gathers the payload and XORs the windows back.  Same outputs as the out-of-place step."""
    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
    pl = ct.make_payloads([synth.payload(args.payload_chars, 7 + i) for i in range(B)], dev)
    work = covers.clone()
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    pay = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)

    def step():
        codec.encode(work, pl, stego=work, maps=maps, meta=meta, check=False)
        codec.decode(work, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words, cover=work,
                     payload=pay)

    for _ in range(args.warmup):
        step()
    el = _timed(torch, dist, world, dev, step, args.steps)
    kern = _profile(_lib.load(), _lib, step, args.steps) if not args.no_profile else {}
    recs = ct.meta_records(meta)
    cover_ok = bool(torch.equal(work.view(torch.int16), covers.view(torch.int16)))
    pay_ok = payload_equal(pay, pl.words, [r.total_used for r in recs])
    status_ok = all(r.status == 0 for r in recs)
    written = sum(r.total_used for r in recs)
    res = {"value": round(B * H * W * world * args.steps / el / 1e6, 1), "unit": "Mpixels/s",
           "ms_per_step": round(el / args.steps * 1e3, 4), "roundtrip_ok": cover_ok and pay_ok and status_ok,
           # every pixel is READ (the decision's histogram/block scan, k_scan_read); only the
           # payload windows are written (embed) and rewritten (restore)
           "value_basis": "pixels read (the whole cover: the scan); written pixels are the windows only",
           "touched_fraction": 1.0, "written_fraction": round(2 * written / (B * H * W), 6),
           "kernels_ms": {k: round(v, 4) for k, v in kern.items()}}
    rk = next((k for k in ("k_scan_rows_read", "k_scan_read") if k in kern), None)
    if rk:   # read-only pass over the cover
        tag = "k_scan_rows" if rk == "k_scan_rows_read" else rk
        res["roofline"] = _roof(rk, B * H * W * 2, kern[rk], pmc_traffic(tag, B, H, W, args.kind, {3: "false"} if tag == "k_scan_rows" else None))
    return res


def bench_c3(args, torch, dist, world, dev, rank):
    """BASELINE config C3: 256 x 512^2 synthetic slices on one GPU (1/16 of the headline
    bytes: 128 MiB per image tensor, so part of each pass can hit the 256 MiB Infinity
    Cache -- reported as measured, against the HBM peak).  The MED-PEE step, and the
    reference's LSB step in `lsb`."""
    B, H, W = 256, 512, 512
    covers = make_covers(torch, args.kind, B, H, W, dev, seed=1000 + rank * B)
    res = {"workload": f"{args.kind} 512x512 uint16 x 256 slices (C3), MED-PEE with capacity control "
                       f"(T = 'auto': a {args.payload_chars}-char payload needs T ~ 4-5 on a 512^2 ct12 slice)"}
    res.update(bench_pee(args, torch, dist, 1, rank, dev, covers, B, H, W, steps=4 * args.steps, T="auto"))
    # unique HBM bytes of the step (cover read + stego write + stego read + cover write) / step time
    res["step_hbm_gbs"] = round(B * H * W * 8 / (res["ms_per_step"] / 1e3) / 1e9, 1)
    lsb = bench_lsb(args, torch, dist, 1, rank, dev, covers, B, H, W, steps=4 * args.steps, seed0=5000)
    lsb.pop("_stego", None)
    res["lsb"] = lsb
    if args.kind == "ct12":   # scheme 2 at T = 2 (a ct12 slice's 1 KB fits in two passes)
        res["pee_scheme2"] = bench_pee2(args, torch, dev, covers, B, H, W, steps=4 * args.steps, T=2)
    return res


def bench_pee2(args, torch, dev, covers, B, H, W, steps, T=2):
    """MED-PEE scheme 2 (four sublattice passes on the running image, oracle/pee_cpu.py) on
    the C3 batch: embed + extract per step at a fixed T (the passes that have bits left run;
    the rest skip their slices), the exact round trip, the passes each slice used, and the
    stego's PSNR (src/mse.py metric, peak 4095 for ct12) beside scheme 1's with capacity
    control on the same payloads."""
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd import quality as Q
    from codec_tcc_amd.pee import PeeCodec
    codec = PeeCodec(B, H, W, dtype="uint16", T=T, maxval=4095, device=dev, scheme=2)
    pay = [synth.payload(args.payload_chars, 99 + i) for i in range(B)]
    packed = codec.pack_payloads(pay)
    stego = torch.empty_like(covers)
    cov2 = torch.empty_like(covers)
    lm = torch.empty((4, B, codec.lm_words), dtype=torch.int64, device=dev)
    meta = torch.empty((4, B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=dev)
    pw = packed[0].shape[1]
    outw = torch.empty((B, pw), dtype=torch.int64, device=dev)
    box = {}

    def step():
        box["enc"] = codec.embed(covers, None, stego=stego, lm=lm, meta=meta, packed=packed, check=False)
        codec.extract(stego, meta, lm, payload_words=pw, cover=cov2, payload=outw)

    for _ in range(args.warmup):
        step()
    el = _timed(torch, None, 1, dev, step, steps)
    enc = box["enc"]
    got = enc.embedded()
    cover_ok = bool(torch.equal(cov2.view(torch.int16), covers.view(torch.int16)))
    pay_ok = payload_equal(outw, packed[0], got)
    full = all(g == n for g, n in zip(got, packed[1]))
    prs = enc.pass_records()
    used = [sum(1 for p in range(4) if prs[p][b].L > 0) for b in range(B)]
    kern = _profile(_lib.load(), _lib, step, steps) if not args.no_profile else {}
    q2 = Q.quality(covers, stego, max_value=4095)
    c1 = PeeCodec(B, H, W, dtype="uint16", T="auto", maxval=4095, device=dev)
    e1 = c1.embed(covers, None, packed=packed)
    q1 = Q.quality(covers, e1.stego, max_value=4095)
    return {"scheme": 2, "T": T, "value": round(B * H * W * steps / el / 1e6, 1), "unit": "Mpixels/s",
            "ms_per_step": round(el / steps * 1e3, 4), "roundtrip_ok": cover_ok and pay_ok and full,
            "cover_ok": cover_ok, "payload_ok": pay_ok, "all_bits_embedded": full,
            "passes_used": {str(n): int(sum(1 for u in used if u == n)) for n in sorted(set(used))},
            "psnr_db_mean": round(float(np.mean([r["psnr"] for r in q2])), 3),
            "pixels_changed_mean": float(np.mean([r["pixels_diferentes"] for r in q2])),
            "scheme1": {"T_chosen": {str(t): int(sum(1 for r in e1.records() if r.T == t))
                                     for t in sorted({r.T for r in e1.records()})},
                        "psnr_db_mean": round(float(np.mean([r["psnr"] for r in q1])), 3),
                        "pixels_changed_mean": float(np.mean([r["pixels_diferentes"] for r in q1]))},
            "kernels_ms": {k: round(v, 4) for k, v in kern.items()},
            "path": "codec_pee_multi_embed / _extract: pass 0 on scheme 1's copy-fused embed, then one "
                    "slice-serial launch per direction for the other passes (the extract with its copy), in "
                    "place on the running image"}


def bench_c4(args, torch, dist, world, rank, dev):
    """BASELINE config C4 at N > 1: 256 x 512^2 ct12 slices per rank (2048 slices on 8 GPUs),
    the MED-PEE step with capacity control and the RCCL all-gather of every slice's side
    information + location-map prefix (PeeRecordExchange, overlapped with extract)."""
    B, H, W = 256, 512, 512
    covers = make_covers(torch, args.kind, B, H, W, dev, seed=3000 + rank * B)
    res = {"workload": f"{args.kind} 512x512 uint16 x {B} slices/GPU x {world} GPUs (C4), MED-PEE T='auto' + "
                       f"all-gather of side information and location maps"}
    res.update(bench_pee(args, torch, dist, world, rank, dev, covers, B, H, W, exchange=True,
                         steps=4 * args.steps, T="auto"))
    return res


def bench_c2(args, torch, dev, rank):
    """BASELINE config C2: ONE 2048^2 slice (a latency case), the MED-PEE step (single pass
    with flat slots over all XCDs at this batch size) and the LSB step, wall clock per step
    over many steps."""
    B, H, W = 1, 2048, 2048
    covers = make_covers(torch, args.kind, B, H, W, dev, seed=7000 + rank)
    res = {"workload": f"{args.kind} 2048x2048 uint16 x 1 slice (C2)"}
    res["pee"] = bench_pee(args, torch, None, 1, rank, dev, covers, B, H, W, steps=10 * args.steps,
                           graph=args.c2_graph)
    lsb = bench_lsb(args, torch, None, 1, rank, dev, covers, B, H, W, steps=10 * args.steps, seed0=7000)
    lsb.pop("_stego", None)
    res["lsb"] = lsb
    return res


def bench_quality(args, torch, covers, stego, B, H, W):
    """Stego quality of a leg's output -- the headline MED-PEE stego (`pee.quality`) and the
    LSB one (`quality`) -- with the reference's src/mse.py metrics: one read-only pass over
    cover + stego (k_quality), metrics from exact moments on the host."""
    from codec_tcc_amd import _lib
    from codec_tcc_amd import quality as Q
    q = Q.quality(covers, stego)
    torch.cuda.synchronize()
    kern = _profile(_lib.load(), _lib, lambda: Q.moments(covers, stego), 5) if not args.no_profile else {}
    res = {"psnr_db_mean": round(float(np.mean([r["psnr"] for r in q])), 3),
           "ssim_min": float(min(r["ssim"] for r in q)),
           "pixels_changed_mean": float(np.mean([r["pixels_diferentes"] for r in q])),
           "kernels_ms": {k: round(v, 4) for k, v in kern.items()}}
    if "k_quality" in kern:
        res["roofline"] = _roof("k_quality", B * H * W * 4, kern["k_quality"],   # read cover + stego
                                pmc_traffic("k_quality", B, H, W, args.kind))
    return res


def _strip_private(d):
    """Drop the `_`-prefixed per-rank fields from a leg's result (recursively)."""
    if isinstance(d, dict):
        return {k: _strip_private(v) for k, v in d.items() if not k.startswith("_")}
    return d


def _device_uuid(props) -> str:
    """The device UUID as hex ('' when the build does not expose it)."""
    u = getattr(props, "uuid", None)
    try:
        return bytes(u.bytes).hex()
    except (AttributeError, TypeError, ValueError):
        return ""


def rank_record(torch, dist, rank, local, dev, backend, head, c4):
    """What this rank ran on: enough for a reader of the N > 1 JSON line
    to check that N ranks ran on N distinct devices over the named backend."""
    p = torch.cuda.get_device_properties(dev)
    import socket
    rec = {"rank": rank, "local_rank": local, "device": dev.index, "pid": os.getpid(),
           "host": socket.gethostname(),
           "pci": f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                  f"{getattr(p, 'pci_device_id', 0):02x}",
           "uuid": _device_uuid(p),   # tells apart partitions sharing one PCI address
           "gpu": p.name, "arch": getattr(p, "gcnArchName", ""),
           "backend": dist.get_backend(), "world_size": dist.get_world_size(),
           "ms_per_step": head.get("_rank_ms_per_step"),
           "kernels_only_ms": head.get("_rank_kernels_only_ms")}
    if c4 is not None:
        rec["c4_ms_per_step"] = c4.get("_rank_ms_per_step")
    return rec


def gather_rank_records(torch, dist, world, rec, backend):
    """Every rank's record, in rank order (one all_gather_object after the timed loops).
    Over RCCL the devices must be distinct (host, PCI address, device UUID -- the UUID tells
    apart compute partitions of one package): RCCL itself refuses two ranks on one GPU, and a
    duplicate here would mean the launcher mapped ranks wrongly."""
    recs = [None] * world
    dist.all_gather_object(recs, rec)
    if backend == "nccl":
        seen = {(r["host"], r["pci"], r.get("uuid", "")) for r in recs}
        if len(seen) != world:
            raise RuntimeError(f"bench.py: {world} RCCL ranks on {len(seen)} distinct devices: {recs}")
    return recs


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


PR_SET_PDEATHSIG = 1      # <linux/prctl.h>


def _die_with_parent(parent_pid: int):
    """preexec_fn of a rank (runs in the child between fork and exec, before any GPU call):
    SIGKILL this process when the launcher dies, however it dies (the flag survives the
    exec).  If the launcher is already gone, exit at once."""
    import ctypes
    import signal
    libc = ctypes.CDLL(None, use_errno=True)
    libc.prctl(PR_SET_PDEATHSIG, int(signal.SIGKILL), 0, 0, 0)
    if os.getppid() != parent_pid:
        os._exit(1)


def _stop_ranks(procs, grace_s: float = 5.0):
    """SIGTERM every live rank, SIGKILL what is still alive after `grace_s`, reap all."""
    for p in procs:
        if p.poll() is None:
            try:
                p.terminate()
            except ProcessLookupError:
                pass
    t_end = time.monotonic() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.0, t_end - time.monotonic()))
        except Exception:   # subprocess.TimeoutExpired
            pass
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait()


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, as torchrun sets them),
    wait for all of them and forward rank 0's JSON line.  This process never touches the GPU
    (no HIP call, no torch.cuda query) and never execs: the ranks are child processes.

    Fail-safe: the ranks stay in this process group (a signal to the
    group reaches them) and get PR_SET_PDEATHSIG = SIGKILL (a killed launcher never leaves
    ranks holding GPUs); SIGTERM/SIGINT here stop every rank and exit non-zero; rank 0's
    output is drained on a thread while every rank is polled, so the first rank that exits
    non-zero -- whichever it is -- stops the others at once (exit status of that failure)."""
    import signal
    import subprocess
    import threading
    n = int(args.gpus)
    env0 = dict(os.environ)
    env0.setdefault("MASTER_ADDR", "127.0.0.1")
    env0["MASTER_PORT"] = str(_free_port()) if "MASTER_PORT" not in os.environ else os.environ["MASTER_PORT"]
    env0["WORLD_SIZE"] = str(n)
    env0["LOCAL_WORLD_SIZE"] = str(n)
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL / cross-process tensors)
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    me = os.getpid()
    procs = []

    def on_signal(signum, _frame):
        _stop_ranks(procs, grace_s=2.0)
        sys.stderr.write(f"bench.py: launcher got signal {signum}; stopped {len(procs)} ranks\n")
        os._exit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    lines = []
    try:
        for r in range(n):
            env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
            # rank 0's stdout is piped (its JSON line is forwarded); the other ranks' stdout goes to
            # stderr, so library chatter (gloo prints its peer count) never reaches stdout
            procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True,
                                          preexec_fn=lambda: _die_with_parent(me)))
        sys.stderr.write("bench.py: rank pids " + " ".join(str(p.pid) for p in procs) + "\n")
        sys.stderr.flush()

        def drain(stream):               # rank 0's output: keep the JSON line, echo the rest
            for raw in stream:
                if raw.startswith("{"):
                    lines.append(raw.strip())
                else:
                    sys.stderr.write(raw)
        reader = threading.Thread(target=drain, args=(procs[0].stdout,), daemon=True)
        reader.start()
        rc = 0
        live = list(procs)
        while live and rc == 0:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = code if code > 0 else 128 - code
                    sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the others\n")
                    break
            time.sleep(0.05)
        reader.join(timeout=10)
    finally:
        _stop_ranks(procs)
        for s, h in old.items():
            signal.signal(s, h)
    line = lines[-1] if lines else None
    if rc == 0 and line:
        print(line, flush=True)
    elif rc == 0:
        sys.stderr.write("bench.py: rank 0 printed no JSON line\n")
        rc = 1
    return rc


def _rank_fault_knob(rank: int):
    """CODEC_BENCH_FAIL_RANK=k (tests of the launcher only): rank k exits 3 right after
    joining the process group; CODEC_BENCH_STALL_RANK=k: rank k sleeps forever there."""
    if os.environ.get("CODEC_BENCH_FAIL_RANK") == str(rank):
        sys.stderr.write(f"bench.py: rank {rank} failing on request (CODEC_BENCH_FAIL_RANK)\n")
        sys.stderr.flush()
        os._exit(3)
    if os.environ.get("CODEC_BENCH_STALL_RANK") == str(rank):
        while True:
            time.sleep(1)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))          # before anything touches the GPU
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (the launcher started a different "
                 "number of ranks)")
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pools = {}
    cpu_base = None
    if args.cpu_seconds > 0 and world == 1:
        # before anything touches the GPU: the baselines run in forked, core-pinned children
        cpu_base = cpu_baseline(args)
        if args.cpu_pool > 0:
            pools["pee"] = cpu_baseline_pool(args, "pee")
            if args.cpu_ref_seconds > 0:
                pools["lsb"] = cpu_baseline_pool(args, "lsb")
    ndev = torch.cuda.device_count()   # counting devices does not initialise the GPU
    if world > 1 and args.backend == "nccl" and ndev < world:
        sys.exit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {ndev} visible "
                 "(--backend gloo rehearses the multi-rank path with several ranks per GPU)")
    if world > 1:
        # a collective that waits longer than this (a dead or stuck peer) raises instead of
        # hanging the job; rank 0's solo legs (C3, quality) stay far below it
        from datetime import timedelta
        pg_timeout = timedelta(seconds=float(os.environ.get("CODEC_BENCH_PG_TIMEOUT", "180")))
        if ndev:
            torch.cuda.set_device(local % ndev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % ndev), timeout=pg_timeout)
        else:   # rehearsal of the multi-rank path on fewer GPUs (e.g. gloo, 2 ranks on 1 GPU)
            dist.init_process_group(args.backend, timeout=pg_timeout)
        _rank_fault_knob(rank)
        dist.barrier()                        # every rank is up before any GPU work
    if ndev == 0:
        sys.exit("bench.py: no GPU visible (the benchmark runs the HIP kernels; there is no CPU path)")
    dev = torch.device("cuda", local % ndev if world > 1 else torch.cuda.current_device())
    B, H, W = args.batch, args.size, args.size
    covers = make_covers(torch, args.kind, B, H, W, dev, seed=rank * B)

    head = bench_pee(args, torch, dist, world, rank, dev, covers, B, H, W, exchange=world > 1)
    pee_stego = head.pop("_stego")
    if rank == 0:   # MED-PEE stego quality (src/mse.py metrics) beside the LSB one
        head["quality"] = bench_quality(args, torch, covers, pee_stego, B, H, W)
    del pee_stego
    inplace = bench_pee(args, torch, dist, world, rank, dev, covers, B, H, W, inplace=True)
    lsb = None
    quality = None
    if args.lsb:
        lsb = bench_lsb(args, torch, dist, world, rank, dev, covers, B, H, W, exchange=world > 1)
        stego = lsb.pop("_stego")
        lsb["inplace"] = bench_lsb_inplace(args, torch, dist, world, dev, covers, B, H, W)
        quality = bench_quality(args, torch, covers, stego, B, H, W) if rank == 0 else None
        del stego
    c4 = bench_c4(args, torch, dist, world, rank, dev) if (world > 1 and args.c3) else None
    ranks = None
    if world > 1:
        ranks = gather_rank_records(torch, dist, world,
                                    rank_record(torch, dist, rank, local, dev, args.backend, head, c4), args.backend)
    c3 = bench_c3(args, torch, dist, world, dev, rank) if (rank == 0 and args.c3) else None
    c2 = bench_c2(args, torch, dev, rank) if (rank == 0 and args.c2 and world == 1) else None

    if rank == 0:
        out = {
            "metric": METRIC, "value": head["value"], "unit": "Mpixels/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
            "data": "synthetic",
            "value_path": "MED-PEE embed + extract (codec_pee_embed / codec_pee_extract, out of place: stego "
                          "and restored cover written in full), the north star's algorithm; the reference has "
                          "no PEE code (SURVEY §0.1), its own bit-plane LSB path is the 'lsb' object",
            "config": {"workload": f"{args.kind} {H}x{W} uint16 x {B} slices/GPU, {args.payload_chars}-char "
                                   f"payload/slice, MED-PEE T={args.pee_T}; embed + extract"
                                   + (f" + {'RCCL' if args.backend == 'nccl' else args.backend} all-gather of "
                                      "per-slice PEE side information + location maps (side stream, overlapped "
                                      "with extract)" if world > 1 else ""),
                       "global_batch": B * world, "slice": f"{H}x{W}", "parallelism": f"slices/{world} GPUs"},
            "roofline": head.get("roofline"),
            "embed_read_roofline_frac": head.get("embed_read_roofline_frac"),
            "step_hbm_gbs": round(B * H * W * 8 / (head["ms_per_step"] / 1e3) / 1e9, 1),
            "kernels_ms": head["kernels_ms"],
            "roundtrip_ok": head["roundtrip_ok"],
            "pee": {k: v for k, v in head.items() if k not in ("value", "ms_per_step", "roofline", "kernels_ms",
                                                                 "roundtrip_ok", "embed_read_roofline_frac")},
            "inplace": inplace,
        }
        if lsb is not None:
            out["lsb"] = lsb
            out["quality"] = quality
        if c3 is not None:
            out["c3"] = c3
        if c4 is not None:
            out["c4"] = c4
        if c2 is not None:
            out["c2"] = c2
        if cpu_base is not None:
            out["cpu_baseline"] = cpu_base
            if "pee" in pools:
                out["cpu_baseline"]["pool"] = pools["pee"]
            if "lsb" in pools and "reference_path" in out["cpu_baseline"]:
                out["cpu_baseline"]["reference_path"]["pool"] = pools["lsb"]
        out = _strip_private(out)
        if ranks is not None:
            out["ranks"] = ranks
            out["distinct_devices"] = len({(r["host"], r["pci"], r.get("uuid", "")) for r in ranks})
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()   # rank 0 ran its C3 leg alone: every rank leaves the group together
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
