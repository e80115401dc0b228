"""Phase stamps of the slice-serial MED-PEE embed (diagnostic build, -DPEE_SS_TRACE).

    python tools/ss_trace.py build          # here: tools/bin/libcodec_sstrace.so
    python tools/ss_trace.py run [inplace]  # GPU box: one embed of 256 x 2048^2, stamps of slice 0

Per chunk k of workgroup 0 (wave 0): t0 chunk start, t1 after classification (the chunk's
pixels have arrived), t2 after the scan barrier, t3 after the stores + refill are issued.
Prints cycles (s_memtime) per phase."""
import ctypes as C
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tools", "bin", "libcodec_sstrace.so")

if sys.argv[1] == "build":
    from codec_tcc_amd import build as B
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    k0 = sys.argv[2] if len(sys.argv) > 2 else "0"   # first traced chunk
    cmd = [B.hipcc(), *B.FLAGS, "-DPEE_SS_TRACE", f"-DPEE_SS_TRACE_K0={k0}", f"-I{B.INC}", *B.SRCS, "-o", OUT]
    subprocess.run(cmd, check=True)
    print(OUT)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from codec_tcc_amd import _lib, synth  # noqa: E402

lib = _lib.load(OUT)
fn = lib.codec_debug_ss_trace
fn.restype = C.c_int
fn.argtypes = [C.c_void_p, C.c_int]
from codec_tcc_amd.pee import PeeCodec  # noqa: E402

inplace = len(sys.argv) > 2 and sys.argv[2] == "inplace"
B, H, W = 256, 2048, 2048
covers = synth.ct12_torch(B, H, W, "cuda", seed=3).view(torch.uint16)
os.environ["CODEC_PEE_SS"] = "1"
pc = PeeCodec(B, H, W, T=2)
packed = pc.pack_payloads([synth.payload(1024, i) for i in range(B)])
for _ in range(3):
    work = covers.clone()
    pc.embed(work if inplace else covers, None, stego=work if inplace else None, packed=packed, check=False)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 2048)()
n = fn(buf, 2048)
t = np.array(buf[:n], dtype=np.uint64).reshape(16, 128).astype(np.float64)
k = 32
t = t[:, : 4 * k].reshape(16, k, 4)
bad = (t[:, :, 2] < t[:, :, 1]) | (t[:, :, 2] > t[:, :, 3])   # no scan stamp (chunk past `end`)
t[:, :, 2] = np.where(bad, t[:, :, 1], t[:, :, 2])
t = t.astype(np.int64)
t0 = t[0, 0, 0]
print(f"{'inplace' if inplace else 'out of place'}: {k} chunks traced (workgroup 0, 16 waves), cycles since the first stamp")
print("chunk  start(w0)  data_min  data_max  barrier_out_min  barrier_out_max  end_max  per_chunk")
for i in range(k):
    st = t[0, i, 0] - t0
    if not t[0, i, 0]:
        continue
    print(f"{i:5d} {st:10d} {t[:, i, 1].min() - t0:9d} {t[:, i, 1].max() - t0:9d} {t[:, i, 2].min() - t0:15d} "
          f"{t[:, i, 2].max() - t0:15d} {t[:, i, 3].max() - t0:8d} {(t[0, i + 1, 0] - t[0, i, 0]) if i + 1 < k else 0:9d}")
print("slowest wave to reach the data per chunk:", [int(np.argmax(t[:, i, 1])) for i in range(k)])
