#!/usr/bin/env python3
"""Small-batch MED-PEE step (embed + extract, out of place) per launch path, HIP-event timed:
flat single pass (default for B < 32), 8-lane single pass, two pass.  Also checks that the
three paths give identical stego / location maps / payload / restored cover.

    python tools/pee_small_batch.py [--size 2048] [--batches 1,2,4,8,16,31]
"""
import argparse
import json
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np
import torch

from codec_tcc_amd import _lib, synth
from codec_tcc_amd.pee import PeeCodec

PATHS = {"flat": {}, "flat_ticket": {"CODEC_PEE_FLAT_TICKET": "1"}, "lanes": {"CODEC_PEE_ONEPASS": "1", "CODEC_PEE_FLAT_MAXB": "0"},
         "twopass": {"CODEC_PEE_ONEPASS": "0"}}
KNOBS = ("CODEC_PEE_ONEPASS", "CODEC_PEE_FLAT_MAXB", "CODEC_PEE_FLAT_TICKET")

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=2048)
ap.add_argument("--batches", default="1,2,4,8,16,31")
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
H = W = a.size
for B in [int(x) for x in a.batches.split(",")]:
    covers = torch.from_numpy(np.stack([synth.ct12(H, W, 500 + i) for i in range(B)])).cuda()
    pay = [synth.payload(1024, 77 + i) for i in range(B)]
    codec = PeeCodec(B, H, W, T=2)
    packed = codec.pack_payloads(pay)
    pw = packed[0].shape[1]
    out, ref = {}, None
    for name, env in PATHS.items():
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)
        stego = torch.empty_like(covers)
        cov2 = torch.empty_like(covers)
        lm = torch.empty((B, codec.lm_words), dtype=torch.int64, device="cuda")
        meta = torch.empty((B, _lib.PEE_META_BYTES), dtype=torch.uint8, device="cuda")
        words = torch.empty((B, pw), dtype=torch.int64, device="cuda")

        def step():
            codec.embed(covers, None, stego=stego, lm=lm, meta=meta, packed=packed)
            codec.extract(stego, meta, lm, payload_words=pw, cover=cov2, payload=words)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            step()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        got = (stego.cpu(), lm.cpu(), words.cpu())
        ok = bool(torch.equal(cov2, covers))
        if ref is None:
            ref = got
        same = all(torch.equal(x, y) for x, y in zip(got, ref))
        out[name] = {"us_per_step": round(us, 1), "roundtrip_ok": ok, "same_as_flat": same,
                     "mpx_s": round(B * H * W / us, 1)}
    for k in KNOBS:
        os.environ.pop(k, None)
    print(json.dumps({"B": B, "size": H, **out}), flush=True)
