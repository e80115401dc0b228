"""k_quality time (HIP events, median of 20 launches) at the bench shape with a given library:
    python tools/quality_time.py tools/bin/libX.so"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from codec_tcc_amd import _lib  # noqa: E402


def main():
    lib = _lib.load(os.path.abspath(sys.argv[1]))
    import torch

    import bench
    from codec_tcc_amd import quality as Q
    dev = torch.device("cuda", 0)
    B, H, W = 256, 2048, 2048
    a = bench.make_covers(torch, "ct12", B, H, W, dev, 0)
    b = a.clone()
    b.view(torch.int16).view(-1)[::97] ^= 1
    Q.moments(a, b)
    torch.cuda.synchronize()
    _lib.check(lib.codec_profile_begin(64), "profile")
    for _ in range(20):
        Q.moments(a, b)
    torch.cuda.synchronize()
    ms = (C.c_float * 64)()
    tags = (C.c_int32 * 64)()
    n = lib.codec_profile_end(ms, tags, 64)
    t = [ms[k] for k in range(n) if _lib.KERNEL_TAGS[tags[k]] == "k_quality"]
    print(f"k_quality {np.median(t):.4f} ms  ({2 * B * H * W * 2 / np.median(t) / 1e9:.2f} TB/s)")


if __name__ == "__main__":
    main()
