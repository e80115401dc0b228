#!/usr/bin/env python3
"""Median duration of each kernel and of the idle gap before it, over the last N launches
of a rocprofv3 kernel trace (one stream): python tools/c2_gaps.py run_kernel_trace.csv [N]"""
import collections
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
rows = rows[-n:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:60]
    dur[name].append((e - s) / 1e3)
    if prev_end is not None:
        gap[name].append((s - prev_end) / 1e3)
    prev_end = e
for k in dur:
    print(f"{k:60s} n={len(dur[k]):4d} dur_us={statistics.median(dur[k]):7.2f} gap_before_us={statistics.median(gap[k]) if gap[k] else 0:7.2f}")
