#!/usr/bin/env python3
"""Event-timing floor of one launch on this box (what a latency leg like C2 pays per kernel):
HIP-event time of a 1-element kernel, of an 8 MiB device copy (a 2048^2 uint16 slice), and of
2 / 3 such copies back to back -- the C2 legs' kernel counts."""
import json

import torch


def timed(fn, reps=200):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1000.0)
    ts.sort()
    return {"median_us": round(ts[len(ts) // 2], 2), "p10_us": round(ts[len(ts) // 10], 2)}


def main():
    dev = torch.device("cuda", 0)
    tiny = torch.zeros(1, device=dev)
    a = torch.randint(0, 4096, (2048, 2048), dtype=torch.int16, device=dev)
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    d = torch.empty_like(a)
    out = {
        "tiny_kernel": timed(lambda: tiny.add_(1)),
        "copy_8MiB": timed(lambda: b.copy_(a)),
        "copy_8MiB_x2": timed(lambda: (b.copy_(a), c.copy_(b))),
        "copy_8MiB_x3": timed(lambda: (b.copy_(a), c.copy_(b), d.copy_(c))),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
