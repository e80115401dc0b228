#!/usr/bin/env python3
"""rocprofv3 kernel trace -> compact per-kernel summary of this build's kernels.

    python tools/prof_summary.py gpurun_out/prof "header line" > profiles/rNN/rocprof_summary.txt

Reads <dir>/run_kernel_trace.csv (one row per dispatch) and prints, per kernel, the mean over
all dispatches and the mean over the dispatches after the first `--skip` of that kernel (the
warm-up launches of bench.py, which the HIP-event figures in bench.json exclude too), so the
two sources can be compared like for like.  Falls back to run_kernel_stats.csv if needed."""
import argparse
import collections
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("header", nargs="?", default="")
ap.add_argument("--skip", type=int, default=2, help="leading dispatches per kernel to drop (warm-up)")
a = ap.parse_args()
print(a.header)
print()
trace = os.path.join(a.dir, "run_kernel_trace.csv")
if os.path.exists(trace):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        n = r["Kernel_Name"]
        if " k_" in n or n.startswith("k_") or "rocclr" in n:
            d[n].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows = []
    for n, v in d.items():
        v.sort()
        us = [x for _, x in v]
        steady = us[a.skip:] if len(us) > a.skip else us
        rows.append((sum(us), n, len(us), sum(us) / len(us), sum(steady) / len(steady), min(us), max(us)))
    print(f"{'kernel':72s} {'calls':>5s} {'avg_us':>9s} {'avg_us(skip %d)' % a.skip:>15s} {'min_us':>9s} {'max_us':>9s}")
    for _, n, c, avg, st, mn, mx in sorted(rows, reverse=True):
        print(f"{n[:72]:72s} {c:5d} {avg:9.2f} {st:15.2f} {mn:9.2f} {mx:9.2f}")
else:
    for r in sorted(csv.DictReader(open(os.path.join(a.dir, "run_kernel_stats.csv"))),
                    key=lambda r: -float(r["TotalDurationNs"])):
        n = r["Name"]
        if " k_" in n or n.startswith("k_") or "rocclr" in n:
            print(f"{n[:72]:72s} calls={int(r['Calls']):4d} avg_us={float(r['AverageNs'])/1e3:9.2f}")
