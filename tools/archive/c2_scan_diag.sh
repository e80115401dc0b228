#!/bin/bash
# C2 LSB scan (k_scan_fast, 1 x 2048^2): histogram cost and workgroup count (HIP events)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 200 python tools/tune.py --batch 1 --size 2048 --rounds 7 --steps 10 --configs \
  '[{}, {"CODEC_DIAG_NOHIST": "1"}, {"CODEC_SCAN_WGS": "32"}, {"CODEC_SCAN_WGS": "64"}, {"CODEC_SCAN_WGS": "256"}, {"CODEC_SCAN_WGS": "32", "CODEC_DIAG_NOHIST": "1"}]' \
  > gpurun_out/c2_scan_diag.log 2>&1; rc=$?
tail -8 gpurun_out/c2_scan_diag.log; exit $rc
