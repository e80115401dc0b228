#!/usr/bin/env python3
"""Scheme-2 MED-PEE embed + extract at C3 (256 x 512^2 ct12, 1 KB, T=2), a few steps, for
rocprofv3 --kernel-trace (per-launch durations of the lattice kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from codec_tcc_amd import _lib, synth  # noqa: E402
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B, H, W = 256, 512, 512
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=1000)
codec = PeeCodec(B, H, W, dtype="uint16", T=2, maxval=4095, device=dev, scheme=2)
packed = codec.pack_payloads([synth.payload(1024, 99 + i) for i in range(B)])
stego = torch.empty_like(covers)
cov2 = torch.empty_like(covers)
lm = torch.empty((4, B, codec.lm_words), dtype=torch.int64, device=dev)
meta = torch.empty((4, B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=dev)
pw = packed[0].shape[1]
outw = torch.empty((B, pw), dtype=torch.int64, device=dev)
for _ in range(int(os.environ.get("STEPS", "6"))):
    codec.embed(covers, None, stego=stego, lm=lm, meta=meta, packed=packed, check=False)
    codec.extract(stego, meta, lm, payload_words=pw, cover=cov2, payload=outw)
torch.cuda.synchronize()
print("roundtrip", bool(torch.equal(cov2, covers)))
