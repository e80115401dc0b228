#!/bin/bash
# column-split k_scan_fast (CODEC_SCAN_CSPLIT / CODEC_SCAN_WGS): LSB GPU parity tests with the
# split forced on every small batch, then C2 / 8-slice timings (HIP events)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for w in 256 2048; do
  CODEC_SCAN_WGS=$w timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py \
      -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/csplit_tests_$w.log 2>&1; rc=$?
  echo "wgs=$w"; tail -1 gpurun_out/csplit_tests_$w.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python tools/tune.py --batch 1 --size 2048 --rounds 7 --steps 10 --configs \
  '[{}, {"CODEC_SCAN_WGS": "256"}, {"CODEC_SCAN_WGS": "512"}, {"CODEC_SCAN_WGS": "256", "CODEC_SCAN_CSPLIT": "4"}]' \
  > gpurun_out/c2_csplit.log 2>&1 || exit 1
tail -4 gpurun_out/c2_csplit.log
timeout -k 10 200 python tools/tune.py --batch 4 --size 2048 --rounds 5 --steps 10 --configs \
  '[{}, {"CODEC_SCAN_WGS": "256"}]' > gpurun_out/c2_csplit_b4.log 2>&1 || exit 1
tail -2 gpurun_out/c2_csplit_b4.log
