"""Phase timing of k_decide's walk path (wide 16-bit slices; diagnostic).  Needs
tools/bin/libcodec_hip_dts.so built with -DDECIDE_TS (see tools/decide_phases.py).  The
covers avoid the top 16 values so the stamps (written to the unused term scratch) never
collide with data.  Stamps: 1 pass 1, 2 terms (skipped), 6 H(Y), 12-15 the first plane's
walk sum (scans, seek, leaves, tree), 7 first plane done, 3 all planes, 4 offset, 5 meta."""
import os, sys
import numpy as np
sys.path.insert(0, "/root/repo")
import torch
from codec_tcc_amd import _lib
_lib.load("/root/repo/tools/bin/libcodec_hip_dts.so")
import bench
import codec_tcc_amd as ct
from codec_tcc_amd import synth
B, H, W = 64, 2048, 2048
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev); g.manual_seed(0)
covers = torch.randint(0, 65520, (B, H, W), generator=g, device=dev, dtype=torch.int32).to(torch.uint16)
codec = ct.Codec(B, H, W, dtype="uint16", device=dev)
pl = ct.make_payloads([synth.payload(1024, 7 + i) for i in range(B)], dev)
for _ in range(3):
    codec.encode(covers, pl)
torch.cuda.synchronize()
R = 65536
keys = (B * R * 4 + 255) // 256 * 256
orv = (keys + B * 8 + 255) // 256 * 256
exact = (orv + B * 4 + 255) // 256 * 256
cap = ((H + 15) // 16) * ((W + 15) // 16)
terms = (exact + B * cap * 8 + 255) // 256 * 256
ws = codec.workspace.cpu().numpy()
raw = ws[terms: terms + B * R * 8].view(np.int64).reshape(B, R)[:, R - 16:]
base = raw[:, 0]
for k in (1, 2, 6, 12, 13, 14, 15, 7, 3, 4, 5):
    print(k, "%.2f us" % (np.median(raw[:, k] - base) * 0.01))
lib = _lib.load()
import time
for _ in range(2):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(5): codec.encode(covers, pl)
    torch.cuda.synchronize(); print("encode ms", (time.perf_counter() - t0) / 5 * 1e3)
