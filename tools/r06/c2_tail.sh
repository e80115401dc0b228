#!/bin/bash
# the scan's last workgroup deciding the slice (k_scan_tail_decide) vs the separate k_decide
# launch, in one process: 1 / 2 / 4 x 2048^2 (C2 and neighbours) + C2 bench legs
export CODEC_TUNING=1
mkdir -p gpurun_out/r06
for b in 1 2 4; do
  timeout -k 10 120 python tools/tune.py --batch $b --size 2048 --rounds 5 --steps 20 \
    --configs '[{}, {"CODEC_SCAN_TAIL_DECIDE": "0"}, {}, {"CODEC_SCAN_TAIL_DECIDE": "0"}]' 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/r06/c2_tail.txt
