#!/usr/bin/env python3
"""Phase timeline of k_pee_embed_res at C3 (256 x 512^2 ct12, T='auto'): per workgroup the
read phase, the T selection, the ranks of the embed phase (pass A + one block scan) and its
items (pass B) (wall_clock64, 100 MHz), from the stamps of a
CODEC_PEE_RES_TRACE=1 run.
    CODEC_PEE_RES_TRACE=1 python3 tools/res_trace.py"""
import ctypes as C
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from codec_tcc_amd import _lib, synth  # noqa: E402
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B, H, W = 256, 512, 512
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=1000)
codec = PeeCodec(B, H, W, dtype="uint16", T="auto", device=dev)
packed = codec.pack_payloads([synth.payload(1024, 99 + i) for i in range(B)])
stego = torch.empty_like(covers)
for _ in range(5):
    enc = codec.embed(covers, None, stego=stego, packed=packed, check=False)
    codec.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
torch.cuda.synchronize()
enc = codec.embed(covers, None, stego=stego, packed=packed, check=False)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (B * 5))()
n = _lib.load().codec_debug_res_trace(buf, B * 5)
t = np.frombuffer(buf, dtype=np.uint64)[: B * 5].astype(np.int64).reshape(B, 5)
t = (t - t[:, 0].min()) * 10 / 1000.0   # us
for name, a, b in (("start", 0, 0), ("read phase", 0, 1), ("select T", 1, 2), ("ranks", 2, 3),
                   ("embed items", 3, 4), ("total", 0, 4)):
    d = t[:, b] - t[:, a] if a != b else t[:, 0]
    print(f"{name:12s} min {d.min():7.2f}  median {np.median(d):7.2f}  max {d.max():7.2f} us")
print("last workgroup ends at %.2f us" % t[:, 4].max())
print("start by slice %% 8 (XCD): " + " ".join("x%d %.2f" % (x, np.median(t[x::8, 0])) for x in range(8)))
