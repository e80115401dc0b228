#!/usr/bin/env python3
"""C3 LSB step (256 x 512^2 ct12: codec_plan + embed + codec_extract) a few times, for
rocprofv3 kernel traces and knob sweeps:  python3 tools/c3_lsb.py [steps]
LSB_SHAPE=BxHxW overrides the shape (e.g. 1x2048x2048 for C2)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import codec_tcc_amd as ct  # noqa: E402
from codec_tcc_amd import synth  # noqa: E402

B, H, W = (int(x) for x in os.environ.get("LSB_SHAPE", "256x512x512").split("x"))
dev = torch.device("cuda", 0)
covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=1000)
codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
pl = ct.make_payloads([synth.payload(1024, 5000 + i) for i in range(B)], dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    enc = codec.encode(covers, pl)
    words, cover = codec.decode(enc.stego, enc.maps, enc.meta, payload_words=pl.payload_words, map_words=pl.map_words)
torch.cuda.synchronize()
print("ok", bool(torch.equal(cover.view(torch.int16), covers.view(torch.int16))))
