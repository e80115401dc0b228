#!/bin/bash
# decision phase stamps (diagnostic -DDECIDE_TS build in tools/r06/lib) at C3, C2 and the
# headline slice size; then the LSB parity suites on the release library.
set -o pipefail
mkdir -p gpurun_out/r06
stop() { echo "stopping after rc $1 ($2)"; exit "$1"; }
export DTS_LIB=tools/r06/lib/libcodec_hip_dts.so
DTS_SIZE=512 DTS_B=256 timeout -k 10 120 python -u tools/decide_phases.py > gpurun_out/r06/phases_c3.txt 2>&1 || stop $? c3
DTS_SIZE=2048 DTS_B=1 timeout -k 10 120 python -u tools/decide_phases.py > gpurun_out/r06/phases_c2.txt 2>&1 || stop $? c2
DTS_SIZE=2048 DTS_B=64 timeout -k 10 120 python -u tools/decide_phases.py > gpurun_out/r06/phases_2048.txt 2>&1 || stop $? h
unset DTS_LIB
cat gpurun_out/r06/phases_c3.txt gpurun_out/r06/phases_c2.txt gpurun_out/r06/phases_2048.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/pytest_lsb.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "^FAILED|^ERROR" gpurun_out/r06/pytest_lsb.log | head -20; tail -2 gpurun_out/r06/pytest_lsb.log
[ $rc -le 1 ] || stop $rc pytest
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
