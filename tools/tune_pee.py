#!/usr/bin/env python3
"""Interleaved A/B of PEE launch knobs (env read per call by the C ABI), out of place and
in place, on the bench workload.

    python tools/tune_pee.py --configs '[{"CODEC_PEE_IP_WGS": "1024"}, {}]' [--rounds 3]
Prints, per configuration and mode, the median per-kernel HIP-event times over rounds."""
import argparse
import json
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="[{}]")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--kind", default="ct12")
    ap.add_argument("--no-check", action="store_true", help="diagnostic builds: skip the round-trip check")
    ap.add_argument("--lib", default=None, help="alternative build of libcodec_hip.so")
    ap.add_argument("--T", default="2", help="PEE threshold, or 'auto' (capacity control, e.g. C3)")
    ap.add_argument("--modes", default="oop,ip", help="comma list of oop (out of place) / ip (in place)")
    a = ap.parse_args()
    import torch
    if a.lib:
        from codec_tcc_amd import _lib
        _lib.load(os.path.abspath(a.lib))

    import bench
    configs = json.loads(a.configs)
    dev = torch.device("cuda", 0)
    B, H, W = a.batch, a.size, a.size
    covers = bench.make_covers(torch, a.kind, B, H, W, dev, 0)
    T = a.T if a.T == "auto" else int(a.T)
    args = types.SimpleNamespace(payload_chars=1024, pee_T=T, warmup=2, steps=10, no_profile=False, kind=a.kind)
    modes = [m == "ip" for m in a.modes.split(",")]
    res = {}
    for _ in range(a.rounds):
        for i, cfg in enumerate(configs):
            saved = {k: os.environ.get(k) for k in cfg}
            os.environ.update(cfg)
            for mode in modes:
                r = bench.bench_pee(args, torch, None, 1, 0, dev, covers, B, H, W, inplace=mode)
                assert a.no_check or r["roundtrip_ok"], (cfg, mode)
                d = res.setdefault((i, mode), {})
                for k, v in r["kernels_ms"].items():
                    d.setdefault(k, []).append(v)
                d.setdefault("step_ms", []).append(r["ms_per_step"])
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    for (i, mode), d in sorted(res.items()):
        print(json.dumps({"cfg": configs[i], "inplace": mode,
                          "ms": {k: round(float(np.median(v)), 4) for k, v in d.items()}}))


if __name__ == "__main__":
    main()
