#!/bin/bash
# C2 (1 x 2048^2) scan: with and without its histogram (CODEC_DIAG_NOHIST: timing only), and
# the column split (csplit 2: 256 workgroups) -- what the lone slice's scan spends on the
# histogram adds + flush
export CODEC_TUNING=1
mkdir -p gpurun_out/r06
timeout -k 10 120 python tools/tune.py --batch 1 --size 2048 --rounds 5 --steps 20 \
  --configs '[{}, {"CODEC_DIAG_NOHIST": "1"}, {"CODEC_SCAN_CSPLIT": "2"}, {}]' 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06/c2_scan_diag.txt
