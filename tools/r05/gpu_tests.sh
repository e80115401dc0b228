#!/bin/bash
# round 5 development loop: the in-place access-pattern ubench, the GPU suite (the new
# workspace / 8-rank tests included) and a short bench.
# Test failures (pytest rc 1) do not stop the later steps; a timeout, abort or crash does.
set -o pipefail
mkdir -p gpurun_out/r05
stop() { echo "stopping after rc $1 ($2)"; exit "$1"; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/ubench_inplace.hip -o /tmp/ubench_inplace || stop 3 hipcc
timeout -k 10 120 /tmp/ubench_inplace > gpurun_out/r05/ubench_inplace.txt 2>&1; rc=$?
echo "ubench rc $rc"; [ $rc -eq 0 ] || stop $rc ubench
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
    > gpurun_out/r05/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "FAILED|ERROR" gpurun_out/r05/pytest_gpu.log | head -30; tail -3 gpurun_out/r05/pytest_gpu.log
[ $rc -le 1 ] || stop $rc pytest
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r05/bench_quick.json 2> gpurun_out/r05/bench_quick.err; rc=$?
echo "bench rc $rc"; [ $rc -eq 0 ] || stop $rc bench
