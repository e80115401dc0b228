#!/usr/bin/env python3
"""Phase timing of k_decide (diagnostic): loads tools/bin/libcodec_hip_dts.so (built with
-DDECIDE_TS, which makes k_decide's thread 0 stamp wall_clock64() at phase boundaries into
its term scratch) and prints median per-phase microseconds over the batch.
    hipcc ... -DDECIDE_TS ... -o tools/bin/libcodec_hip_dts.so && python tools/decide_phases.py"""
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    from codec_tcc_amd import _lib
    _lib.load(os.environ.get("DTS_LIB", os.path.join(REPO, "tools", "bin", "libcodec_hip_dts.so")))
    import bench
    import codec_tcc_amd as ct
    from codec_tcc_amd import synth
    kind = sys.argv[1] if len(sys.argv) > 1 else "ct12"
    B = int(os.environ.get("DTS_B", "64"))
    H = W = int(os.environ.get("DTS_SIZE", "2048"))
    dev = torch.device("cuda", 0)
    covers = bench.make_covers(torch, kind, B, H, W, dev, 0)
    codec = ct.Codec(B, H, W, dtype="uint16", device=dev)
    pl = ct.make_payloads([synth.payload(1024, 7 + i) for i in range(B)], dev)
    for _ in range(3):
        codec.encode(covers, pl)
    torch.cuda.synchronize()
    if os.environ.get("DTS_ISOLATED") == "1":   # the stamped call alone on an idle GPU
        import time
        time.sleep(0.05)
        codec.encode(covers, pl)
        torch.cuda.synchronize()
    R = 65536
    keys = (B * R * 4 + 255) // 256 * 256
    orv = (keys + B * 8 + 255) // 256 * 256
    slots = (orv + B * 4 + 255) // 256 * 256
    exact = (slots + B * 16 * 8 + 255) // 256 * 256
    nby = (H + 15) // 16
    cap = nby * ((W + 15) // 16)
    terms = (exact + B * cap * 8 + 255) // 256 * 256
    ws = codec.workspace.cpu().numpy()
    raw = ws[terms: terms + B * R * 8].view(np.int64).reshape(B, R)[:, R - 16:]
    t = raw[:, :6]
    split = B * 17 <= 240 and os.environ.get("CODEC_DECIDE_SPLIT", "1") != "0"
    if split:   # plane workgroups: entry, after pass 1 + terms, after the list, after the sum
        pr = ws[terms: terms + B * R * 8].view(np.int64).reshape(B, R)[:, R - 80:R - 16].reshape(B, 16, 4)
        t0 = raw[:, 0:1]
        act = pr[:, :, 3] > pr[:, :, 2]
        print("split: plane start %.2f us after main, pass1+terms %.2f, list %.2f, sum %.2f, last plane done %.2f us "
              "after main start; main: H(Y) done %.2f, collect done %.2f us" % (
                  np.median(pr[:, :, 0] - t0) * 0.01, np.median((pr[:, :, 1] - pr[:, :, 0])) * 0.01,
                  np.median((pr[:, :, 2] - pr[:, :, 1])[act]) * 0.01, np.median((pr[:, :, 3] - pr[:, :, 2])[act]) * 0.01,
                  np.median(np.max(np.where(act, pr[:, :, 3], pr[:, :, 1]), axis=1) - t0[:, 0]) * 0.01,
                  np.median(raw[:, 8] - raw[:, 0]) * 0.01, np.median(raw[:, 14] - raw[:, 0]) * 0.01))
    w0 = raw[:, 6:8] if not split else None   # wave 0 (plane 0): after its H(X,Y) sum, after its joint-order list
    if not split:   # per-wave end of the first round's plane (wave 15: H(Y)), after the round start (DTS 2)
        wvt = ws[terms: terms + B * R * 8].view(np.int64).reshape(B, R)[:, R - 80:R - 64]
        ok = wvt > raw[:, 2:3]
        print("wave path, per wave (us after the MI round start; median over slices): " + " ".join(
            "w%d=%.2f" % (w, np.median((wvt[:, w] - raw[:, 2])[ok[:, w]]) * 0.01) for w in range(16) if ok[:, w].any()))
    # the paired MI round (default) does not stamp wave 0's list/sum slots: skip the breakdown then
    if not split and (w0 > raw[:, 2:3]).all() and (raw[:, 9] >= raw[:, 8]).all(): print("wave0: masks %.2f us, counts+scans %.2f us, list %.2f us, sum %.2f us, then to round end %.2f us" % (
        np.median(raw[:, 8] - raw[:, 2]) * 0.01, np.median(raw[:, 9] - raw[:, 8]) * 0.01,
        np.median(w0[:, 1] - raw[:, 9]) * 0.01, np.median(w0[:, 0] - w0[:, 1]) * 0.01,
        np.median(raw[:, 3] - w0[:, 0]) * 0.01))
    print("pass1 split: loads+pops %.2f us, block scan %.2f us, pop reductions %.2f us" % (
        np.median(raw[:, 12] - raw[:, 0]) * 0.01, np.median(raw[:, 13] - raw[:, 12]) * 0.01,
        np.median(raw[:, 1] - raw[:, 13]) * 0.01))
    d = np.diff(t, axis=1)
    names = ["pass1+scan", "terms", "H(Y)+MI", "offset argmax", "windows/meta"]
    med = np.median(d, axis=0)
    print(kind, "wall_clock64 ticks (100 MHz => 10 ns/tick):")
    for n, v in zip(names, med):
        print(f"  {n:16s} {v:8.0f} ticks = {v * 0.01:7.2f} us")
    print(f"  total            {np.median(t[:, -1] - t[:, 0]) * 0.01:7.2f} us")
    t00 = t[:, 0].min()
    print("slices' entry stamps: median %.2f, max %.2f us after the first; last decision done %.2f us, last embed "
          "done %.2f us after the first entry" % (np.median(t[:, 0] - t00) * 0.01, (t[:, 0].max() - t00) * 0.01,
                                                  (t[:, -1].max() - t00) * 0.01, (raw[:, 11].max() - t00) * 0.01))
    if (raw[:, 15] > 0).all() and os.environ.get("DTS_SIZE") == "512":   # fused kernel: workgroup start stamps
        st = raw[:, 15]
        scan = (t[:, 0] - st) * 0.01
        print("fused: workgroup starts spread %.2f us; scan (start -> decision entry) median %.2f, min %.2f, max %.2f us"
              % ((st.max() - st.min()) * 0.01, np.median(scan), scan.min(), scan.max()))
        print("  by slice % 8 (the XCD its workgroup is dealt to): " + " ".join(
            "x%d: start %.2f scan %.2f" % (x, np.median(st[x::8] - st.min()) * 0.01, np.median(scan[x::8])) for x in range(8)))
        order = np.argsort(t[:, 0])
        print("  slowest 8 slices (scan us): " + " ".join("b%d=%.1f" % (i, scan[i]) for i in order[-8:]))
    print("embed (fused): load_win %.2f us, embed loop %.2f us" % (np.median(raw[:, 10] - raw[:, 5]) * 0.01,
                                                                np.median(raw[:, 11] - raw[:, 10]) * 0.01))


if __name__ == "__main__":
    main()
