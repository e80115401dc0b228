#!/bin/bash
# the whole GPU suite, fast-decision phase stamps, a quick bench
set -o pipefail
mkdir -p gpurun_out/r06
stop() { echo "stopping after rc $1 ($2)"; exit "$1"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "^FAILED|^ERROR" gpurun_out/r06/pytest_gpu.log | head -20; tail -2 gpurun_out/r06/pytest_gpu.log
[ $rc -le 1 ] || stop $rc pytest
: > gpurun_out/r06/fast_phases.txt
bash tools/r06/fast_phases.sh || stop $? phases
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --cpu-ref-seconds 0 \
    > gpurun_out/r06/bench_quick.json 2> gpurun_out/r06/bench_quick.err; rc=$?
echo "bench rc $rc"; [ $rc -eq 0 ] || stop $rc bench
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06/bench_quick.json").read().strip().splitlines()[-1])
l = d.get("lsb", {}); c3 = d.get("c3", {}).get("lsb", {}); c2 = d.get("c2", {}).get("lsb", {})
print("headline", d["value"], d["ms_per_step"])
for n, x in (("lsb", l), ("c3.lsb", c3), ("c2.lsb", c2)):
    print(n, x.get("ms_per_step"), x.get("roundtrip_ok"), x.get("decide"), x.get("kernels_ms"))
PY
