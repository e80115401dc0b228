#!/bin/bash
# round 5: the GPU suite (the new workspace / 8-rank tests included), then a short bench
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/r05/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r05/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r05/pytest_gpu.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r05/bench_quick.json 2> gpurun_out/r05/bench_quick.err
echo "bench rc $?"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/ubench_inplace.hip -o /tmp/ubench_inplace && \
timeout -k 10 120 /tmp/ubench_inplace > gpurun_out/r05/ubench_inplace.txt 2>&1; echo "ubench rc $?"
timeout -k 10 300 python tools/tune_pee.py --configs '[{}, {"CODEC_PEE_SS_CHAIN": "1"}]' --rounds 5 --modes ip > gpurun_out/r05/chain_ab.txt 2>&1; echo "chain ab rc $?"; cat gpurun_out/r05/chain_ab.txt | tail -4
