#!/bin/bash
# partial histograms for small 16-bit batches (CODEC_SCAN_PARTS): C2 (1 x 2048^2) and 2 / 4
# slices, on vs off (off = one histogram per slice, csplit 1), in one process
export CODEC_TUNING=1
mkdir -p gpurun_out/r06
for b in 1 2 4; do
  timeout -k 10 120 python tools/tune.py --batch $b --size 2048 --rounds 5 --steps 20 \
    --configs '[{}, {"CODEC_SCAN_PARTS": "0"}, {"CODEC_SCAN_PARTS": "0", "CODEC_SCAN_CSPLIT": "2"}, {}]' 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/r06/c2_parts.txt
