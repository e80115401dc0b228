#!/usr/bin/env python3
"""rocprofv3 --kernel-trace CSV -> per-kernel summary (calls, mean, mean without the first
`skip` warm-up launches, min, max) for profiles/rNN/rocprof_summary.txt.
    python tools/rocprof_summary.py gpurun_out/prof/run_kernel_trace.csv "<header line>" [skip]"""
import collections
import csv
import sys

path, header = sys.argv[1], sys.argv[2]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 2
runs = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if name.startswith("void at::") or "elementwise" in name or "reduce_kernel" in name:
        continue
    runs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(header)
print()
print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'avg_us(skip %d)' % skip:>15s} {'min_us':>9s} {'max_us':>9s}")
for name, v in sorted(runs.items(), key=lambda kv: -sum(kv[1]) / len(kv[1]) * min(len(kv[1]), 22)):
    tail = v[skip:] or v
    print(f"{name[:72]:72s} {len(v):6d} {sum(v) / len(v):9.2f} {sum(tail) / len(tail):15.2f} {min(v):9.2f} {max(v):9.2f}")
