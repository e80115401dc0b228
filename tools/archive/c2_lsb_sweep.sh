#!/bin/bash
# C2 LSB (1 x 2048^2) launch-shape sweep: restore threads / workgroups, the fused gather,
# scan workgroups (HIP events per kernel, tools/tune.py)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune.py --batch 1 --size 2048 --rounds 7 --steps 10 --configs \
  '[{}, {"CODEC_RESTORE_GS_THREADS": "256"}, {"CODEC_RESTORE_GS_THREADS": "512"},
    {"CODEC_RESTORE_GS_THREADS": "256", "CODEC_RESTORE_GS_WGS": "256"},
    {"CODEC_FUSED_GATHER": "0"}, {"CODEC_SCAN_WGS": "64"}, {"CODEC_HIST_MEMSET": "1"}]' \
  > gpurun_out/c2_lsb_sweep.log 2>&1 || exit 1
tail -8 gpurun_out/c2_lsb_sweep.log
