"""Start spread of the fused C3 scan+decide workgroups (diagnostic builds with DECIDE_TS; with
DECIDE_TS_SCAN_ONLY the kernel returns after the scan): workgroup starts per XCD, scan times."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from codec_tcc_amd import _lib
    _lib.load(os.path.abspath(sys.argv[1]))
    import bench
    import codec_tcc_amd as ct
    from codec_tcc_amd import synth
    B, H = 256, 512
    dev = torch.device("cuda", 0)
    covers = bench.make_covers(torch, "ct12", B, H, H, dev, 0)
    codec = ct.Codec(B, H, H, dtype="uint16", device=dev)
    pl = ct.make_payloads([synth.payload(1024, 7 + i) for i in range(B)], dev)
    R = 65536
    keys = (B * R * 4 + 255) // 256 * 256
    orv = (keys + B * 8 + 255) // 256 * 256
    slots = (orv + B * 4 + 255) // 256 * 256
    exact = (slots + B * 16 * 8 + 255) // 256 * 256
    cap = ((H + 15) // 16) ** 2
    terms = (exact + B * cap * 8 + 255) // 256 * 256
    for mode in ("back-to-back", "isolated"):
        for _ in range(3):
            codec.encode(covers, pl, check=False)
        torch.cuda.synchronize()
        if mode == "isolated":
            import time
            time.sleep(0.05)
            codec.encode(covers, pl, check=False)
            torch.cuda.synchronize()
        ws = codec.workspace.cpu().numpy()
        raw = ws[terms: terms + B * R * 8].view(np.int64).reshape(B, R)[:, R - 16:]
        st, en = raw[:, 15], raw[:, 0]
        scan = (en - st) * 0.01
        print("%s: starts spread %.2f us; by XCD %s; scan median %.2f, max %.2f us; last scan end %.2f us after first start" % (
            mode, (st.max() - st.min()) * 0.01,
            " ".join("%.2f" % (np.median(st[x::8] - st.min()) * 0.01) for x in range(8)),
            np.median(scan), scan.max(), (en.max() - st.min()) * 0.01))


if __name__ == "__main__":
    main()
