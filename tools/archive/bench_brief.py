#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line: python tools/bench_brief.py gpurun_out/bench.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = d.get


def leg(name, x):
    if not x:
        return
    roof = (x.get("roofline") or {}).get("frac")
    print(f"{name:10s} {x.get('ms_per_step')} ms  {x.get('kernels_ms')}  frac={roof}  ok={x.get('roundtrip_ok')}")


print(f"headline   {g('value')} {g('unit')}  {g('ms_per_step')} ms  frac={g('roofline', {}).get('frac')}  "
      f"ok={g('roundtrip_ok')}  kernels={g('kernels_ms')}")
leg("inplace", g("inplace"))
leg("lsb", g("lsb"))
leg("lsb.inpl", (g("lsb") or {}).get("inplace"))
leg("c3", g("c3"))
leg("c3.lsb", (g("c3") or {}).get("lsb"))
leg("c2.pee", (g("c2") or {}).get("pee"))
leg("c2.lsb", (g("c2") or {}).get("lsb"))
cb = g("cpu_baseline") or {}
print("cpu", cb.get("value"), cb.get("unit"), "| ref", (cb.get("reference_path") or {}).get("value"))
