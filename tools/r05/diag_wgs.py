"""Diagnose the out-of-place one-pass MED-PEE with a persistent grid (CODEC_PEE_1P_WGS):
bench_pee's round trip at the headline shape, with the fields that decide roundtrip_ok."""
import json
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    B = int(os.environ.get("DIAG_B", "256"))
    H = W = 2048
    covers = bench.make_covers(torch, "ct12", B, H, W, dev, 0)
    args = types.SimpleNamespace(payload_chars=1024, pee_T=2, warmup=1, steps=2, no_profile=True, kind="ct12")
    for wgs in sys.argv[1:]:
        if wgs == "default":
            os.environ.pop("CODEC_PEE_1P_WGS", None)
        else:
            os.environ["CODEC_PEE_1P_WGS"] = wgs
        r = bench.bench_pee(args, torch, None, 1, 0, dev, covers, B, H, W, inplace=False)
        keep = {k: r.get(k) for k in ("roundtrip_ok", "cover_ok", "payload_ok", "lookback_ok", "overflow_slices",
                                      "repaired_slices", "end_candidates_mean", "kernels_ms")}
        print(wgs, json.dumps(keep), flush=True)


if __name__ == "__main__":
    main()
