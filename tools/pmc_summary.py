#!/usr/bin/env python3
"""rocprofv3 --pmc CSVs (gpurun_out/pmc_FETCH_SIZE, pmc_WRITE_SIZE) -> per-kernel HBM bytes
per launch, written to profiles/pmc_traffic.json (read by bench.py) and a round copy.

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports exactly half the bytes of
a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Counters are in KB.
    python tools/pmc_summary.py r01 [--batch 256 --h 2048 --w 2048 --kind ct12]"""
import argparse
import collections
import csv
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("round")
ap.add_argument("--src", default="gpurun_out")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--h", type=int, default=2048)
ap.add_argument("--w", type=int, default=2048)
ap.add_argument("--kind", default="ct12")
ap.add_argument("--name", default="pmc_traffic", help="output file stem (e.g. pmc_traffic_c3)")
ap.add_argument("--prefix", default="pmc", help="input directory prefix under --src (pmc_FETCH_SIZE ...)")
a = ap.parse_args()
vals = {}
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(a.src, f"{a.prefix}_{C}", "run_counter_collection.csv"))):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if name.startswith("k_"):      # keyed per template instantiation (copy vs in place differ)
            agg[name].append(float(r["Counter_Value"]))
    vals[C] = {k: sum(v) / len(v) for k, v in agg.items()}
out = {"config": {"batch": a.batch, "h": a.h, "w": a.w, "kind": a.kind},
       "source": f"profiles/{a.round}/{a.name}.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
       "kernels": {}}
for k in vals["FETCH_SIZE"]:
    f_kb = vals["FETCH_SIZE"][k]
    w_kb = vals["WRITE_SIZE"].get(k, 0.0)
    out["kernels"][k] = {"fetch_size_kb": f_kb, "write_size_kb": w_kb,
                         "hbm_bytes_per_launch": int(round((2 * f_kb + w_kb) * 1024))}
os.makedirs(os.path.join("profiles", a.round), exist_ok=True)
for path in (os.path.join("profiles", a.round, a.name + ".json"), os.path.join("profiles", a.name + ".json")):
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
