#!/usr/bin/env python3
"""Benchmark of the LSB bit-plane embed+extract hot path on MI355X.

One step = encode (codec_plan: histogram/decision/block-search scan + stego copy,
codec_embed: window writes + location maps) + decode (codec_extract: cover restore
stream + payload gather) over one batch of synthetic uint16 slices that are already
resident in HBM, plus (N > 1) the RCCL all-gather of the per-slice records and
location maps (on a side stream after encode, overlapped with decode).  Prints ONE JSON
line (rank 0).

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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event pass")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    ap.add_argument("--pee", type=int, default=1, help="also time the MED-PEE path (north-star algorithm)")
    ap.add_argument("--pee-T", type=int, default=2)
    ap.add_argument("--cpu-pool", type=int, default=16,
                    help="workers of the pooled CPU baseline (the box's CPU share per GPU is 16; 0 = skip)")
    ap.add_argument("--c3", type=int, default=1, help="also time BASELINE config C3 (256 x 512^2)")
    ap.add_argument("--c2", type=int, default=1, help="also time BASELINE config C2 (1 x 2048^2, latency)")
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


def pmc_traffic(kernel: str, b: int, h: int, w: int, kind: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_summary.py: FETCH_SIZE x2 (gfx950 correction)
    + WRITE_SIZE, KB -> bytes), when it was collected on this exact configuration."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    cfg = d.get("config", {})
    if (cfg.get("batch"), cfg.get("h"), cfg.get("w"), cfg.get("kind")) != (b, h, w, kind):
        return None
    ks = d.get("kernels", {})
    k = ks.get(kernel)
    if not k:   # keyed per template instantiation: accept the unique one of this kernel
        hits = [v for n, v in ks.items() if n.split("<")[0] == kernel]
        if len(hits) != 1:
            return None
        k = hits[0]
    return {"hbm_bytes_per_launch": k["hbm_bytes_per_launch"], "source": d.get("source", path)}


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


def cpu_baseline(size: int, kind: str, chars: int, budget_s: float):
    """The oracle (numpy restatement of the reference, bit-identical to it) timed on this
    host: decomposition + hybrid embed + merge + extract_local_planes + decode_message
    (SURVEY §8(d)), single process, on distinct synthetic slices until the budget is used."""
    from codec_tcc_amd import synth
    from oracle import ref_cpu as R
    gen = synth.GENERATORS[kind]
    px = 0
    n = 0
    t_work = 0.0
    t_start = time.perf_counter()
    while n == 0 or (time.perf_counter() - t_start) < budget_s:
        img = gen(size, size, 1000 + n)
        bits = R.message_to_bits(synth.payload(chars, 7 + n))
        t0 = time.perf_counter()
        enc = R.encode_slice(img, bits, beta=0.4, sb=16)
        R.decode_slice(enc["stego"], enc["bitmaps"], enc["s"], enc["segments_lengths"], enc["segment_indices"])
        t_work += time.perf_counter() - t0
        px += img.size
        n += 1
    return {
        "value": round(px / t_work / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
        "sample": f"{n} x {size}x{size} {kind} uint16 slices, {chars}-char payloads, numpy oracle "
                  f"(decompose+hybrid embed+merge+extract_local_planes+decode_message), 1 process",
        "seconds": round(t_work, 2), "cpu_model": _cpu_model(),
    }


def _cpu_slice(job):
    """One oracle encode+decode of a distinct slice (pool worker of cpu_baseline_pool)."""
    size, kind, chars, seed = job
    from codec_tcc_amd import synth
    from oracle import ref_cpu as R
    img = synth.GENERATORS[kind](size, size, seed)
    bits = R.message_to_bits(synth.payload(chars, 7 + seed))
    t0 = time.perf_counter()
    enc = R.encode_slice(img, bits, beta=0.4, sb=16)
    R.decode_slice(enc["stego"], enc["bitmaps"], enc["s"], enc["segments_lengths"], enc["segment_indices"])
    return img.size, time.perf_counter() - t0


def cpu_baseline_pool(size: int, kind: str, chars: int, workers: int, per_worker: int):
    """The same oracle work spread over a process pool (one worker per host core
    of this GPU's share).  Forked BEFORE the GPU is initialised in this process."""
    import multiprocessing as mp
    jobs = [(size, kind, chars, 2000 + i) for i in range(workers * per_worker)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_slice, jobs, chunksize=1)
    wall = time.perf_counter() - t0
    px = sum(r[0] for r in res)
    return {"value": round(px / wall / 1e6, 3), "unit": "Mpixels/s", "cores": workers, "kind": "port",
            "sample": f"{len(jobs)} x {size}x{size} {kind} slices over a {workers}-process pool (fork), wall clock",
            "seconds": round(wall, 2), "cpu_model": _cpu_model()}


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


def bench_lsb_inplace(args, torch, dist, world, dev, covers, codec, pl, B, H, W):
    """The reference-algorithm step in place: codec_plan only reads the cover (no stego copy),
    codec_embed rewrites the <= payload-size window pixels of the same buffer, codec_extract
    gathers the payload and XORs the windows back.  Same outputs as the out-of-place step."""
    from codec_tcc_amd import _lib
    work = covers.clone()
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    pay = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)

    def step():
        codec.encode(work, pl, stego=work, maps=maps, meta=meta)
        codec.decode(work, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words, cover=work,
                     payload=pay)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kern = _profile(_lib.load(), _lib, step, args.steps) if not args.no_profile else {}
    ok = bool(torch.equal(work.view(torch.int16), covers.view(torch.int16)))
    res = {"value": round(B * H * W * world * args.steps / el / 1e6, 1), "unit": "Mpixels/s",
           "ms_per_step": round(el / args.steps * 1e3, 4), "roundtrip_ok": ok,
           "kernels_ms": {k: round(v, 4) for k, v in kern.items()}}
    rk = next((k for k in ("k_scan_rows_read", "k_scan_read") if k in kern), None)
    if rk:
        by = B * H * W * 2                               # read-only pass over the cover
        t_k = kern[rk] / 1e3
        res["roofline"] = {"bound": "hbm", "kernel": rk, "achieved": round(by / t_k / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(by / t_k / 1e9 / HBM_PEAK_GBS, 4),
                           "algorithmic_bytes_per_launch": by}
    return res


def bench_pee(args, torch, dist, world, dev, covers, B, H, W, inplace=False):
    """MED-PEE embed + extract over the same resident batch (1 KB payload per slice).
    Out of place (default): k_pee_embed1 (one pass: copy + look-back cursor + embed) and
    k_pee_extract1 (one pass: copy + look-back cursor + recover).  In place: the same
    kernels read and write only the chunks up to each slice's `end`."""
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd.pee import PeeCodec, PeeEncoded
    codec = PeeCodec(B, H, W, dtype="uint16", T=args.pee_T, device=dev)
    pay = [synth.payload(args.payload_chars, 99 + i) for i in range(B)]
    packed = codec.pack_payloads(pay)
    work = covers.clone() if inplace else None
    stego = work if inplace else torch.empty_like(covers)
    cov2 = work if inplace else torch.empty_like(covers)
    src = work if inplace else covers
    lm = torch.empty((B, codec.lm_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=dev)
    pw = packed[0].shape[1]
    outw = torch.empty((B, pw), dtype=torch.int64, device=dev)

    def step():
        codec.embed(src, None, stego=stego, lm=lm, meta=meta, packed=packed)
        codec.extract(stego, meta, lm, payload_words=pw, cover=cov2, payload=outw)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    recs = PeeEncoded(stego, lm, meta, packed[1], pw).records()
    ok = bool(torch.equal(cov2.view(torch.int16), covers.view(torch.int16))) and all(r.status == 0 for r in recs)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kern = _profile(_lib.load(), _lib, step, args.steps) if not args.no_profile else {}
    ok = ok and bool(torch.equal(cov2.view(torch.int16), covers.view(torch.int16)))
    res = {"value": round(B * H * W * world * args.steps / el / 1e6, 1), "unit": "Mpixels/s",
           "ms_per_step": round(el / args.steps * 1e3, 4), "T": args.pee_T, "roundtrip_ok": ok,
           "end_candidates_mean": float(np.mean([r.end + 1 for r in recs])),
           # slices whose payload exceeds the T-capacity (truncated, still exactly reversible;
           # roundtrip_ok then reads False): uniform-noise slices at T=2
           "overflow_slices": int(sum(1 for r in recs if r.status == 1)),
           "kernels_ms": {k: round(v, 4) for k, v in kern.items()}}
    if inplace:
        # algorithmic bytes: every 8-px x 2-row item up to the one holding `end` is read
        # (candidates + their neighbours), its candidate row written back
        prefix_px = sum(((r.end // 4) + 1) * 16 for r in recs if r.end >= 0)
        by = prefix_px * 2 + prefix_px // 2 * 2
        res["algorithmic_bytes_per_step_half"] = by
        t_e = kern.get("k_pee_embed1", 0.0) / 1e3
        if t_e > 0:
            tr = pmc_traffic("k_pee_embed1<unsigned short, true, true>", B, H, W, getattr(args, "kind", "ct12"))
            res["roofline"] = {"bound": "hbm", "kernel": "k_pee_embed1", "achieved": round(by / t_e / 1e9, 1),
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(by / t_e / 1e9 / HBM_PEAK_GBS, 4),
                               "traffic": tr["hbm_bytes_per_launch"] if tr else None,
                               "algorithmic_bytes_per_launch": by}
        return res
    for kname in ("k_pee_embed1", "k_pee_scan"):
        if kname in kern:
            t_k = kern[kname] / 1e3
            by = B * H * W * 4
            tr = pmc_traffic(kname + "<unsigned short, true, false>" if kname == "k_pee_embed1" else kname,
                             B, H, W, getattr(args, "kind", "ct12"))
            res["roofline"] = {"bound": "hbm", "kernel": kname, "achieved": round(by / t_k / 1e9, 1),
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(by / t_k / 1e9 / HBM_PEAK_GBS, 4),
                               "traffic": tr["hbm_bytes_per_launch"] if tr else None,
                               "algorithmic_bytes_per_launch": by}
            break
    t_emb = sum(kern.get(k, 0.0) for k in ("k_pee_embed1", "k_pee_scan", "k_pee_locate", "k_pee_embed")) / 1e3
    if t_emb > 0:
        res["embed_read_roofline_frac"] = round(B * H * W * 2 / t_emb / 1e9 / HBM_PEAK_GBS, 4)
    return res


def bench_c3(args, torch, dist, world, dev, rank):
    """BASELINE config C3: the same LSB step over 256 x 512^2 ct12 slices (1/16 of the
    headline bytes: 128 MiB per image tensor, so part of each pass can hit the 256 MiB
    Infinity Cache -- reported as measured, against the HBM peak)."""
    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    B, H, W = 256, 512, 512
    covers = make_covers(torch, args.kind, B, H, W, dev, seed=1000 + rank * B)
    codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
    pl = ct.make_payloads([synth.payload(args.payload_chars, 5000 + rank * B + i) for i in range(B)], dev)
    stego = torch.empty_like(covers)
    cov2 = torch.empty_like(covers)
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    pay = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)

    def step():
        codec.encode(covers, pl, stego=stego, maps=maps, meta=meta)
        codec.decode(stego, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words, cover=cov2,
                     payload=pay)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    steps = 4 * args.steps
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern = _profile(_lib.load(), _lib, step, steps) if not args.no_profile else {}
    ok = bool(torch.equal(cov2.view(torch.int16), covers.view(torch.int16)))
    res = {"workload": f"{args.kind} 512x512 uint16 x 256 slices (C3)", "value": round(B * H * W * steps / el / 1e6, 1),
           "unit": "Mpixels/s", "ms_per_step": round(el / steps * 1e3, 4), "roundtrip_ok": ok,
           "kernels_ms": {k: round(v, 4) for k, v in kern.items()}}
    sk = next((k for k in ("k_scan_rows", "k_scan_fast") if k in kern), None)
    if sk:
        by = B * H * W * 4
        res["roofline"] = {"bound": "hbm", "kernel": sk, "achieved": round(by / (kern[sk] / 1e3) / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(by / (kern[sk] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                           "algorithmic_bytes_per_launch": by}
    return res


def bench_c2(args, torch, dev, rank):
    """BASELINE config C2: ONE 2048^2 ct12 slice (a latency case: one workgroup's worth of
    decisions, a handful of launches).  The LSB step and the MED-PEE step (two-pass path at
    this batch size) timed separately, wall clock per step over many steps."""
    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd.pee import PeeCodec
    B, H, W = 1, 2048, 2048
    covers = make_covers(torch, args.kind, B, H, W, dev, seed=7000 + rank)
    codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
    pl = ct.make_payloads([synth.payload(args.payload_chars, 7000 + rank)], dev)
    stego = torch.empty_like(covers)
    cov2 = torch.empty_like(covers)
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    pay = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)
    pc = PeeCodec(B, H, W, dtype="uint16", T=args.pee_T, device=dev)
    packed = pc.pack_payloads([synth.payload(args.payload_chars, 7100 + rank)])
    lm = torch.empty((B, pc.lm_words), dtype=torch.int64, device=dev)
    pmeta = torch.empty((B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=dev)
    pw = packed[0].shape[1]
    pout = torch.empty((B, pw), dtype=torch.int64, device=dev)
    pst = torch.empty_like(covers)
    pcov = torch.empty_like(covers)

    def lsb():
        codec.encode(covers, pl, stego=stego, maps=maps, meta=meta)
        codec.decode(stego, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words, cover=cov2,
                     payload=pay)

    def pee():
        pc.embed(covers, None, stego=pst, lm=lm, meta=pmeta, packed=packed)
        pc.extract(pst, pmeta, lm, payload_words=pw, cover=pcov, payload=pout)

    res = {"workload": f"{args.kind} 2048x2048 uint16 x 1 slice (C2)"}
    steps = 10 * args.steps
    for name, fn, outc in (("lsb", lsb, cov2), ("pee", pee, pcov)):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern = _profile(_lib.load(), _lib, fn, steps) if not args.no_profile else {}
        res[name] = {"ms_per_step": round(el / steps * 1e3, 4), "value": round(H * W * steps / el / 1e6, 1),
                     "unit": "Mpixels/s", "roundtrip_ok": bool(torch.equal(outc.view(torch.int16), covers.view(torch.int16))),
                     "kernels_ms": {k: round(v, 4) for k, v in kern.items()}}
    return res


def bench_quality(args, torch, covers, stego, B, H, W):
    """Stego quality of the LSB leg's output (reference src/mse.py metrics): one read-only
    pass over cover + stego (k_quality), metrics from exact moments on the host."""
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
        by = B * H * W * 4                                # read cover + read stego (uint16)
        t_k = kern["k_quality"] / 1e3
        res["roofline"] = {"bound": "hbm", "kernel": "k_quality", "achieved": round(by / t_k / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(by / t_k / 1e9 / HBM_PEAK_GBS, 4),
                           "algorithmic_bytes_per_launch": by}
    return res


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pool_base = None
    if args.cpu_seconds > 0 and world == 1 and args.cpu_pool > 0:
        # before anything touches the GPU: the pool forks this process
        pool_base = cpu_baseline_pool(args.size, args.kind, args.payload_chars, args.cpu_pool, 2)
    ndev = torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local % ndev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % ndev))
        else:   # rehearsal of the multi-rank path on fewer GPUs (e.g. gloo, 2 ranks on 1 GPU)
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local % ndev if world > 1 else torch.cuda.current_device())
    B, H, W = args.batch, args.size, args.size

    covers = make_covers(torch, args.kind, B, H, W, dev, seed=rank * B)
    msgs = [synth.payload(args.payload_chars, 7 + rank * B + i) for i in range(B)]
    codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
    pl = ct.make_payloads(msgs, dev)
    # preallocated outputs (the step allocates nothing)
    stego = torch.empty((B, H, W), dtype=torch.uint16, device=dev)
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    cover_out = torch.empty((B, H, W), dtype=torch.uint16, device=dev)
    payload_out = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)
    # per-slice fixed-size records (slice meta + packed location map) -> every rank; they
    # depend on encode only, so the all-gather runs on a side stream beside decode
    xch = D.RecordExchange(B, pl.map_words, world, dev) if world > 1 else None
    gathered = xch.gathered if world > 1 else None

    def step():
        codec.encode(covers, pl, stego=stego, maps=maps, meta=meta)
        if world > 1:
            xch.mark()
        codec.decode(stego, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words,
                     cover=cover_out, payload=payload_out)
        if world > 1:
            xch.start(meta, maps)
            xch.join()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness spot check of the warm state (cheap, outside the timed region)
    ok = bool(torch.equal(cover_out.view(torch.int16), covers.view(torch.int16)))
    if world > 1:   # this rank's rows of the gathered records are its own packed records
        ok = ok and bool(torch.equal(gathered[rank * B:(rank + 1) * B], D.pack_records(meta, maps)))

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- N > 1: the all-gather alone and the step without it (kernel-only
    # scaling and the collective reported separately), same barrier + max-over-ranks timing
    dist_split = None
    if world > 1:
        def timed(fn):
            dist.barrier()
            torch.cuda.synchronize()
            t_a = time.perf_counter()
            for _ in range(args.steps):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            tt = torch.tensor([time.perf_counter() - t_a], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            return float(tt.item()) / args.steps

        def gather_only():
            xch.start(meta, maps)
            xch.join()

        def kernels_only():
            codec.encode(covers, pl, stego=stego, maps=maps, meta=meta)
            codec.decode(stego, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words,
                         cover=cover_out, payload=payload_out)

        t_g = timed(gather_only)
        t_k = timed(kernels_only)
        dist_split = {"allgather_ms": round(t_g * 1e3, 4),
                      "allgather_bytes": int(gathered.numel() * gathered.element_size()),
                      "kernels_only_ms_per_step": round(t_k * 1e3, 4),
                      "kernels_only_value": round(B * H * W * world / t_k / 1e6, 1)}

    # ---- per-kernel device time (HIP events on the launch stream), separate timed pass
    kernels = {}
    if not args.no_profile:
        lib = _lib.load()
        cap = 64 * args.steps
        _lib.check(lib.codec_profile_begin(cap), "codec_profile_begin")
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        import ctypes as C
        ms = (C.c_float * cap)()
        tags = (C.c_int32 * cap)()
        n = lib.codec_profile_end(ms, tags, cap)
        for i in range(max(n, 0)):
            kernels.setdefault(_lib.KERNEL_TAGS.get(tags[i], str(tags[i])), []).append(ms[i])

    quality = bench_quality(args, torch, covers, stego, B, H, W) if rank == 0 else None
    c3 = bench_c3(args, torch, dist, world, dev, rank) if (rank == 0 and args.c3) else None
    c2 = bench_c2(args, torch, dev, rank) if (rank == 0 and args.c2 and world == 1) else None
    lsb_inplace = bench_lsb_inplace(args, torch, dist, world, dev, covers, codec, pl, B, H, W)
    pee = None
    if args.pee:
        pee = bench_pee(args, torch, dist, world, dev, covers, B, H, W)
        pee["inplace"] = bench_pee(args, torch, dist, world, dev, covers, B, H, W, inplace=True)

    npx_rank = B * H * W
    total_px = npx_rank * world
    ms_step = elapsed / args.steps * 1e3
    value = total_px * args.steps / elapsed / 1e6

    recs = ct.meta_records(meta)
    s_vals = sorted({r.s for r in recs})
    roof = None
    sk = next((k for k in ("k_scan_rows", "k_scan_fast") if k in kernels), None)
    if sk:
        t_scan = float(np.mean(kernels[sk])) / 1e3
        bytes_scan = npx_rank * (2 + 2)              # read cover + write stego (uint16)
        ach = bytes_scan / t_scan / 1e9
        roof = {"bound": "hbm", "kernel": sk, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "algorithmic_bytes_per_launch": bytes_scan, "avg_launch_ms": round(t_scan * 1e3, 4)}
        tr = pmc_traffic(sk, B, H, W, getattr(args, "kind", "ct12"))
        if tr is not None:
            roof["traffic"] = tr["hbm_bytes_per_launch"]
            roof["traffic_source"] = tr["source"]
    step_bytes = npx_rank * 8                        # cover r + stego w + stego r + cover w
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mpixels/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
            "data": "synthetic",
            "value_path": "the reference's pixel path (bit-plane LSB embed + true decode, src/codec.py:412-487, "
                          "752-793), bit-exact; the north star's MED-PEE embed+extract on the same batch is the "
                          "'pee' object (the reference has no PEE code, SURVEY §0.1)",
            "config": {"workload": f"{args.kind} {H}x{W} uint16 x {B} slices/GPU, {args.payload_chars}-char "
                                   f"payload/slice, beta=0.4, block=16; encode(plan+embed)+decode(restore+gather)"
                                   + (f" + {'RCCL' if args.backend == 'nccl' else args.backend} all-gather of slice records/maps (side stream, overlapped with decode)"
                                      if world > 1 else ""),
                       "global_batch": B * world, "slice": f"{H}x{W}", "parallelism": f"slices/{world} GPUs"},
            "roofline": roof,
            "step_hbm_gbs": round(step_bytes * world / (elapsed / args.steps) / 1e9 / world, 1),
            "kernels_ms": {k: round(float(np.mean(v)), 4) for k, v in kernels.items()},
            "s_values": s_vals,
            "roundtrip_ok": ok,
        }
        if dist_split is not None:
            out["distributed"] = dist_split
        out["inplace"] = lsb_inplace
        out["quality"] = quality
        if c3 is not None:
            out["c3"] = c3
        if c2 is not None:
            out["c2"] = c2
        if pee is not None:
            out["pee"] = pee
        if args.cpu_seconds > 0 and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.size, args.kind, args.payload_chars, args.cpu_seconds)
            if pool_base is not None:
                out["cpu_baseline"]["pool"] = pool_base
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
