#!/usr/bin/env python3
"""C3 MED-PEE step (256 x 512^2 ct12, T='auto') a few times, for rocprofv3 kernel traces:
    rocprofv3 --kernel-trace --stats -d gpurun_out/c3 -o run -- python3 tools/c3_pee.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from codec_tcc_amd import synth  # noqa: E402
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B, H, W = 256, 512, 512
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=1000)
codec = PeeCodec(B, H, W, dtype="uint16", T="auto", device=dev)
packed = codec.pack_payloads([synth.payload(1024, 99 + i) for i in range(B)])
stego = torch.empty_like(covers)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    enc = codec.embed(covers, None, stego=stego, packed=packed, check=False)
    codec.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
torch.cuda.synchronize()
print("ok", codec.repaired(enc.payload_words))
