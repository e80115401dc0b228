#!/bin/bash
# round 5: the GPU suite (the new workspace / 8-rank tests included), then a short bench
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r05/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r05/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r05/pytest_gpu.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r05/bench_quick.json 2> gpurun_out/r05/bench_quick.err
echo "bench rc $?"
