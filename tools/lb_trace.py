"""Phase stamps of the look-back single-pass MED-PEE embed (diagnostic build, -DPEE_LB_TRACE).

    python tools/lb_trace.py build          # here: tools/bin/libcodec_lbtrace.so
    python tools/lb_trace.py run [B]        # GPU box: embed of B x 2048^2 (default 1), per-slot phases

Per slot (workgroup iteration), thread 0's s_memtime at: 0 slot start, 1 after the ticket /
finished-flag barrier, 2 after classification + block scan, 3 after the look-back barrier,
4 after the embed, 5 after the stores are issued.  Prints percentiles of each phase and the
spread of slot starts / ends (ramp and tail), in shader-clock cycles."""
import ctypes as C
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tools", "bin", "libcodec_lbtrace.so")

if sys.argv[1] == "build":
    from codec_tcc_amd import build as B
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run([B.hipcc(), *B.FLAGS, "-DPEE_LB_TRACE", f"-I{B.INC}", *B.SRCS, "-o", OUT], check=True)
    print(OUT)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from codec_tcc_amd import _lib, synth  # noqa: E402

lib = _lib.load(OUT)
fn = lib.codec_debug_lb_trace
fn.restype = C.c_int
fn.argtypes = [C.c_void_p, C.c_int]
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
H = W = 2048
covers = synth.ct12_torch(B, H, W, "cuda", seed=3).view(torch.uint16)
pc = PeeCodec(B, H, W, T=2)
packed = pc.pack_payloads([synth.payload(1024, i) for i in range(B)])
stego = torch.empty_like(covers)
for _ in range(5):
    pc.embed(covers, None, stego=stego, packed=packed, check=False)
torch.cuda.synchronize()
nslots = min(4096, B * 256)
buf = (C.c_ulonglong * (nslots * 12))()
fn(buf, nslots * 12)
t = np.array(buf[:], dtype=np.uint64).reshape(nslots, 12).astype(np.float64)
full = t[:, 10] == 0
act = full & (t[:, 7] > t[:, 6]) & (t[:, 8] >= t[:, 7])
t0 = t[:, 0].min()
print(f"B={B}: {nslots} slots, {int(full.sum())} embedding, {int((~full).sum())} copy-only; cycles")
for name, a, b in [("ticket/flag", 0, 1), ("classify+scan", 1, 2), ("look-back", 2, 3), ("embed", 3, 4), ("stores", 4, 5)]:
    d = (t[full, b] - t[full, a]) if a != 0 or b != 1 else (t[:, b] - t[:, a])
    if d.size:
        print(f"  {name:14s} p10 {np.percentile(d, 10):8.0f}  p50 {np.percentile(d, 50):8.0f}  p90 {np.percentile(d, 90):8.0f}")
for name, a, b in [("meta+barrier", 3, 6), ("embed loop", 6, 7), ("block sum", 7, 8)]:
    d = t[act, b] - t[act, a]
    if d.size:
        print(f"  {name:14s} p10 {np.percentile(d, 10):8.0f}  p50 {np.percentile(d, 50):8.0f}  p90 {np.percentile(d, 90):8.0f}  (active chunks: {int(act.sum())})")
print(f"  slot start spread {t[:, 0].max() - t0:.0f}, last stores issued at {t[:, 5].max() - t0:.0f}, "
      f"first at {t[:, 5].min() - t0:.0f}")
