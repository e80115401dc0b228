#!/usr/bin/env python3
"""C2 MED-PEE step (1 x 2048^2 ct12, T=2, 1 KB) repeated, for rocprofv3 traces / knob sweeps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from codec_tcc_amd import synth  # noqa: E402
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B, H, W = 1, 2048, 2048
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=7000)
codec = PeeCodec(B, H, W, dtype="uint16", T=2, device=dev)
packed = codec.pack_payloads([synth.payload(1024, 99)])
stego = torch.empty_like(covers)
out = torch.empty_like(covers)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 50):
    enc = codec.embed(covers, None, stego=stego, packed=packed, check=False)
    codec.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words, cover=out)
torch.cuda.synchronize()
print("ok", bool(torch.equal(out.view(torch.int16), covers.view(torch.int16))))
