#!/usr/bin/env python3
"""C2 LSB (1 x 2048^2 ct12): the decode's restore launch shape, alternating in one process.
k_restore_gs with 1024-thread workgroups (the default for sweeps <= 512 MiB: 128 workgroups
for a lone 2048^2 slice, half the CUs) against 256-thread ones (512 workgroups) and the
slice-serial kernel; decode time per call (HIP events around codec.decode) and the whole
encode + decode step, every variant's cover and payload checked."""
import os
import sys
import time

os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import codec_tcc_amd as ct  # noqa: E402
from codec_tcc_amd import synth  # noqa: E402

B, H, W = int(os.environ.get("B", "1")), 2048, 2048
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=7000)
codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
pl = ct.make_payloads([synth.payload(1024, 7000 + i) for i in range(B)], dev)
VARIANTS = {"gs1024": {}, "gs256": {"CODEC_RESTORE_GS_THREADS": "256"}}
KEYS = ("CODEC_RESTORE_GS_THREADS",)
lenc = codec.encode(covers, pl, check=True)
ref_words = None


def decode(name):
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(VARIANTS[name])
    return codec.decode(lenc.stego, lenc.maps, lenc.meta, payload_words=pl.payload_words, map_words=pl.map_words)


ok = {}
for name in VARIANTS:
    w, back = decode(name)
    torch.cuda.synchronize()
    if ref_words is None:
        ref_words = w.clone()
    ok[name] = bool(torch.equal(back, covers)) and bool(torch.equal(w, ref_words))
print("check", ok, flush=True)
res = {n: [] for n in VARIANTS}
steps = 50
for rep in range(5):
    for name in VARIANTS:
        decode(name)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            codec.encode(covers, pl, check=False)
            decode(name)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / steps * 1e3)
for name, v in res.items():
    v = sorted(v)
    print(f"{name:8s} encode+decode ms median {v[len(v) // 2]:.4f} min {v[0]:.4f}", flush=True)
