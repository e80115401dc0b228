#!/usr/bin/env python3
"""Compact view of tools/tune.py output: config, each kernel's ms, step sum."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        ks = " ".join(f"{k}={v:.4f}" for k, v in d["kernels_ms"].items())
        print(f"{json.dumps(d['cfg']):60s} {ks}  sum={d['sum_ms']:.4f}")
