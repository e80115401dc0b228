#!/bin/bash
# LSB parity suites on the release library, then the tail-decision A/B (tools/r06/c2_tail.sh)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py tests/test_gpu_tuning.py -m gpu -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/pytest_lsb.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "^FAILED|^ERROR" gpurun_out/r06/pytest_lsb.log | head; tail -1 gpurun_out/r06/pytest_lsb.log
[ $rc -eq 0 ] || exit $rc
bash tools/r06/c2_tail.sh
