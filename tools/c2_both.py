#!/usr/bin/env python3
"""BASELINE C2 (1 x 2048^2 ct12) in one process: the MED-PEE step (T = 2, flat look-back
slots) and the LSB step (codec_encode + codec_extract), a few times each -- for rocprofv3
kernel-trace / PMC passes (tools/c2_pmc.sh):  python3 tools/c2_both.py [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import codec_tcc_amd as ct  # noqa: E402
from codec_tcc_amd import synth  # noqa: E402
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B, H, W = 1, 2048, 2048
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=7000)
pee = PeeCodec(B, H, W, dtype="uint16", T=2, device=dev)
packed = pee.pack_payloads([synth.payload(1024, 99)])
stego = torch.empty_like(covers)
for _ in range(n):
    enc = pee.embed(covers, None, stego=stego, packed=packed, check=False)
    _w, back = pee.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
pl = ct.make_payloads([synth.payload(1024, 7000)], dev)
for _ in range(n):
    lenc = codec.encode(covers, pl, check=False)
    _w2, back2 = codec.decode(lenc.stego, lenc.maps, lenc.meta, payload_words=pl.payload_words,
                              map_words=pl.map_words)
torch.cuda.synchronize()
print("ok", bool(torch.equal(back.view(torch.int16), covers.view(torch.int16))),
      bool(torch.equal(back2.view(torch.int16), covers.view(torch.int16))))
