#!/usr/bin/env python3
"""Per-kernel average durations from a rocprofv3 SQLite output (run_results.db): name, calls,
average (first 2 calls skipped when there are more than 4), min, max in microseconds."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
d = collections.defaultdict(list)
for name, start, end in c.execute("select name, start, end from kernels"):
    d[name].append((end - start) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v2 = v[2:] if len(v) > 4 else v
    print(f"{k[:90]:90s} n={len(v):4d} avg={sum(v2) / len(v2):9.2f} min={min(v):8.2f} max={max(v):8.2f} us")
