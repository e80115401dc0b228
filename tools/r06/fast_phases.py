#!/usr/bin/env python3
"""Phase stamps of the guard-banded (fast) decision, from a -DDECIDE_TS build (DTS_LIB):
entry -> pass 1 loads (12) -> rank scan (13) -> pop reductions (1) -> terms (8) -> exact-H(Y)
leaves + H(Y) partials (6, thread 0) -> barrier (7) -> wave 0 combine / wave 1 walk / wave 2
offset (per-wave stamps) -> barrier (9) -> (2) -> offset/windows (3, 4, 5) -> embed (10, 11).
    DTS_LIB=tools/r06/lib/libcodec_hip_dts.so DTS_SIZE=512 DTS_B=256 python tools/r06/fast_phases.py"""
import os
import sys

import numpy as np

os.environ.setdefault("CODEC_TUNING", "1")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    import torch
    from codec_tcc_amd import _lib
    _lib.load(os.environ["DTS_LIB"])
    import bench
    import codec_tcc_amd as ct
    from codec_tcc_amd import synth
    B = int(os.environ.get("DTS_B", "256"))
    H = W = int(os.environ.get("DTS_SIZE", "512"))
    dev = torch.device("cuda", 0)
    covers = bench.make_covers(torch, "ct12", B, H, W, dev, 0)
    codec = ct.Codec(B, H, W, dtype="uint16", device=dev)
    pl = ct.make_payloads([synth.payload(1024, 7 + i) for i in range(B)], dev)
    for _ in range(3):
        codec.encode(covers, pl)
    torch.cuda.synchronize()
    R = 65536
    keys = (B * R * 4 + 255) // 256 * 256
    orv = (keys + B * 8 + 255) // 256 * 256
    slots = (orv + B * 4 + 255) // 256 * 256
    exact = (slots + B * 16 * 8 + 255) // 256 * 256
    cap = ((H + 15) // 16) * ((W + 15) // 16)
    terms = (exact + B * cap * 8 + 255) // 256 * 256
    ws = codec.workspace.cpu().numpy()
    allr = ws[terms: terms + B * R * 8].view(np.int64).reshape(B, R)
    raw = allr[:, R - 16:]
    wv = allr[:, R - 80:R - 64]
    d = lambda a, b: np.median(raw[:, b] - raw[:, a]) * 0.01
    print(f"B={B} {H}x{W}: pass1 loads {d(0, 12):.2f}, rank scan {d(12, 13):.2f}, pops {d(13, 1):.2f}, "
          f"terms {d(1, 8):.2f}, leaves+partials {d(8, 6):.2f}, barrier {d(6, 7):.2f}, "
          f"after-barrier tasks {d(7, 9):.2f} (wave0 combine {np.median(wv[:, 0] - raw[:, 7]) * 0.01:.2f}, "
          f"wave1 walk {np.median(wv[:, 1] - raw[:, 7]) * 0.01:.2f}, wave2 offset {np.median(wv[:, 2] - raw[:, 7]) * 0.01:.2f}), "
          f"to DTS2 {d(9, 2):.2f}, H(Y)/offset {d(2, 3):.2f}, ->4 {d(3, 4):.2f}, windows {d(4, 5):.2f}, "
          f"embed {d(5, 11):.2f}; decision total {d(0, 5):.2f} us")
    ph = allr[:, R - 112:R - 80].reshape(B, 2, 16)
    if (ph > 0).all():   # per-wave ends of pass 1 and of the terms, relative to the entry stamp
        rel = (ph - raw[:, 0:1, None]) * 0.01
        print("  per wave, median over slices (us after entry): pass 1 end " +
              " ".join(f"{np.median(rel[:, 0, w]):.2f}" for w in range(16)) +
              "; terms end " + " ".join(f"{np.median(rel[:, 1, w]):.2f}" for w in range(16)))


if __name__ == "__main__":
    main()
