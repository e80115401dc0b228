#!/usr/bin/env python3
"""Interleaved in-process A/B of launch-shape knobs (env read per launch by the C ABI).

    python tools/tune.py [--kind ct12] [--rounds 3]
Prints, per configuration, the median per-kernel HIP-event time over rounds."""
import argparse
import ctypes as C
import json
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = [
    {"CODEC_NT": "0", "CODEC_SCAN_WGS": "256", "CODEC_RESTORE_WGS": "2048"},
    {"CODEC_NT": "1", "CODEC_SCAN_WGS": "256", "CODEC_RESTORE_WGS": "2048"},
    {"CODEC_NT": "0", "CODEC_SCAN_WGS": "256", "CODEC_RESTORE_WGS": "32768"},
    {"CODEC_NT": "1", "CODEC_SCAN_WGS": "256", "CODEC_RESTORE_WGS": "32768"},
    {"CODEC_NT": "1", "CODEC_SCAN_WGS": "512", "CODEC_RESTORE_WGS": "32768"},
    {"CODEC_NT": "1", "CODEC_SCAN_WGS": "1024", "CODEC_RESTORE_WGS": "32768"},
    {"CODEC_NT": "1", "CODEC_SCAN_WGS": "2048", "CODEC_RESTORE_WGS": "32768"},
    {"CODEC_NT": "1", "CODEC_SCAN_WGS": "256", "CODEC_RESTORE_WGS": "8192"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="ct12")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--configs", default="")
    ap.add_argument("--inplace", action="store_true", help="stego is cover, cover_out is stego")
    a = ap.parse_args()
    import torch

    import bench
    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    configs = json.loads(a.configs) if a.configs else CONFIGS
    dev = torch.device("cuda", 0)
    B, H, W = a.batch, a.size, a.size
    covers = bench.make_covers(torch, a.kind, B, H, W, dev, 0)
    codec = ct.Codec(B, H, W, dtype="uint16", device=dev)
    pl = ct.make_payloads([synth.payload(1024, 7 + i) for i in range(B)], dev)
    stego = torch.empty_like(covers)
    cov2 = torch.empty_like(covers)
    maps = torch.empty((B, pl.map_words), dtype=torch.int64, device=dev)
    meta = torch.empty((B, _lib.META_BYTES), dtype=torch.uint8, device=dev)
    pay = torch.empty((B, pl.payload_words), dtype=torch.int64, device=dev)
    lib = _lib.load()

    def step():
        codec.encode(covers, pl, stego=stego, maps=maps, meta=meta, check=False)
        codec.decode(stego, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words, cover=cov2,
                     payload=pay)

    def enc():
        codec.encode(covers, pl, stego=stego, maps=maps, meta=meta, check=False)

    if a.inplace:
        work = covers.clone()
        enc = None   # an in-place encode alone would leave the buffer embedded

        def step():   # noqa: F811
            codec.encode(work, pl, stego=work, maps=maps, meta=meta, check=False)
            codec.decode(work, maps, meta, payload_words=pl.payload_words, map_words=pl.map_words, cover=work,
                         payload=pay)
        cov2 = work

    res = {i: {} for i in range(len(configs))}
    keys = {k for cfg in configs for k in cfg}
    for _r in range(a.rounds):
        for i, cfg in enumerate(configs):
            for k in keys:          # a key absent from this config falls back to the default
                os.environ.pop(k, None)
            os.environ.update(cfg)
            step()
            torch.cuda.synchronize()
            cap = 32 * a.steps
            _lib.check(lib.codec_profile_begin(cap), "profile")
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            ms = (C.c_float * cap)()
            tags = (C.c_int32 * cap)()
            n = lib.codec_profile_end(ms, tags, cap)
            per = {}
            for k in range(n):
                per.setdefault(_lib.KERNEL_TAGS[tags[k]], []).append(ms[k])
            for k, v in per.items():
                res[i].setdefault(k, []).append(float(np.mean(v)))
            # wall time of the step and of its encode half (no profile window: launch gaps included)
            for name, fn in (("step_ms", step), ("encode_ms", enc)):
                if fn is None:
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.steps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[i].setdefault(name, []).append(e0.elapsed_time(e1) / a.steps)
    if not torch.equal(cov2.view(torch.int16), covers.view(torch.int16)):   # diagnostic configs (CODEC_DIAG_*)
        print("WARNING: round trip not exact under the last configuration", flush=True)
    for i, cfg in enumerate(configs):
        row = {k: round(float(np.median(v)), 4) for k, v in res[i].items()}
        wall = {k: row.pop(k) for k in ("step_ms", "encode_ms") if k in row}
        tot = round(sum(row.values()), 4)
        print(json.dumps({"cfg": cfg, "kernels_ms": row, "sum_ms": tot, **wall}))


if __name__ == "__main__":
    main()
