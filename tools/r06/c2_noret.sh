#!/bin/bash
# LSB parity suites, then the no-return LDS histogram adds (CODEC_SCAN_NORET) on/off in one
# process: 1 / 2 / 4 x 2048^2
set -o pipefail
mkdir -p gpurun_out/r06
export CODEC_TUNING=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/pytest_lsb.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "^FAILED|^ERROR" gpurun_out/r06/pytest_lsb.log | head; tail -1 gpurun_out/r06/pytest_lsb.log
[ $rc -eq 0 ] || exit $rc
for b in 1 2 4; do
  timeout -k 10 120 python tools/tune.py --batch $b --size 2048 --rounds 5 --steps 20 \
    --configs '[{}, {"CODEC_SCAN_NORET": "0"}, {}, {"CODEC_SCAN_NORET": "0"}]' 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/r06/c2_noret.txt
