#!/usr/bin/env python3
"""rocprofv3 --stats CSV -> compact per-kernel summary (this build's kernels + copies/fills).
    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv "header line" > profiles/rNN/rocprof_summary.txt"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2] if len(sys.argv) > 2 else "")
print()
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = r["Name"]
    if not (" k_" in n or n.startswith("k_") or "rocclr" in n):
        continue
    print(f"{n[:72]:72s} calls={int(r['Calls']):4d} avg_us={float(r['AverageNs'])/1e3:9.2f} "
          f"min_us={float(r['MinNs'])/1e3:9.2f} max_us={float(r['MaxNs'])/1e3:9.2f}")
