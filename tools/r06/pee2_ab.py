#!/usr/bin/env python3
"""Scheme-2 MED-PEE at C3 (256 x 512^2 ct12, 1 KB, T=2): step time (embed + extract) of the
per-pass tile launches (CODEC_PEE_LAT_SS=0) against the slice-serial launch (=1; pass 0 through
scheme 1's kernels, or with CODEC_PEE_LAT_SS_P0=0 every pass in the one launch), alternating in
one process; every variant's stego, records, maps, payload and cover compared with the first."""
import os
import sys
import time

os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from codec_tcc_amd import _lib, synth  # noqa: E402
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B, H, W = int(os.environ.get("B", "256")), 512, 512
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=1000)
codec = PeeCodec(B, H, W, dtype="uint16", T=2, maxval=4095, device=dev, scheme=2)
packed = codec.pack_payloads([synth.payload(1024, 99 + i) for i in range(B)])
pw = packed[0].shape[1]
VARIANTS = {"tile": {"CODEC_PEE_LAT_SS": "0"},
            "ss_p0s1": {"CODEC_PEE_LAT_SS": "1", "CODEC_PEE_LAT_SS_P0": "1"},
            "ss_all": {"CODEC_PEE_LAT_SS": "1", "CODEC_PEE_LAT_SS_P0": "0"},
            "ss_nopf": {"CODEC_PEE_LAT_SS": "1", "CODEC_PEE_LAT_SS_P0": "1", "CODEC_PEE_LAT_SS_PF": "0"}}
bufs = {}
for name in VARIANTS:
    bufs[name] = dict(stego=torch.empty_like(covers), cov=torch.empty_like(covers),
                      lm=torch.zeros((4, B, codec.lm_words), dtype=torch.int64, device=dev),
                      meta=torch.zeros((4, B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=dev),
                      out=torch.empty((B, pw), dtype=torch.int64, device=dev))


def step(name):
    for k in ("CODEC_PEE_LAT_SS", "CODEC_PEE_LAT_SS_P0", "CODEC_PEE_LAT_SS_PF"):
        os.environ.pop(k, None)
    for k, v in VARIANTS[name].items():
        os.environ[k] = v
    b = bufs[name]
    codec.embed(covers, None, stego=b["stego"], lm=b["lm"], meta=b["meta"], packed=packed, check=False)
    codec.extract(b["stego"], b["meta"], b["lm"], payload_words=pw, cover=b["cov"], payload=b["out"])


for name in VARIANTS:
    step(name)
torch.cuda.synchronize()
ref = bufs["tile"]
ok = {}
for name, b in bufs.items():
    recs_ok = True
    for p in range(4):
        mr = ref["meta"][p].cpu().numpy().view("int32").reshape(B, -1)
        mb = b["meta"][p].cpu().numpy().view("int32").reshape(B, -1)
        # L, end, status, T, lattice and lm_count equal; capacity may be partial (flags)
        for col in (0, 2, 3, 6, 7, 9, 13):
            recs_ok &= bool((mr[:, col] == mb[:, col]).all())
    ok[name] = dict(stego=bool(torch.equal(b["stego"], ref["stego"])), cover=bool(torch.equal(b["cov"], covers)),
                    payload=bool(torch.equal(b["out"], packed[0])), records=recs_ok)
print("check", ok, flush=True)
steps = int(os.environ.get("STEPS", "20"))
res = {n: [] for n in VARIANTS}
for rep in range(int(os.environ.get("REPS", "5"))):
    for name in VARIANTS:
        step(name)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(name)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / steps * 1e3)
for name, v in res.items():
    v = sorted(v)
    print(f"{name:10s} step ms median {v[len(v) // 2]:.4f} min {v[0]:.4f} all {[round(x, 4) for x in v]}", flush=True)
