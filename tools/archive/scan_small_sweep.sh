#!/bin/bash
# k_scan_fast workgroup count for small batches (1-8 slices of 2048^2), HIP events
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for B in 1 2 4 8; do
  timeout -k 10 200 python tools/tune.py --batch $B --size 2048 --rounds 5 --steps 10 --configs \
    '[{"CODEC_SCAN_WGS": "128"}, {"CODEC_SCAN_WGS": "256"}, {"CODEC_SCAN_WGS": "512"}]' > gpurun_out/scan_small_$B.log 2>&1 || exit 1
  echo "B=$B"; tail -3 gpurun_out/scan_small_$B.log
done
