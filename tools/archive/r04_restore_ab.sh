#!/bin/bash
# A/B: slice-serial restore with a per-slice rotated start (CODEC_RESTORE_SS_ROT) at the
# headline shape (256 x 2048^2) and at C3 (256 x 512^2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/tune.py --rounds 5 --steps 5 --configs '[{},{"CODEC_RESTORE_SS":"1"},{"CODEC_RESTORE_SS":"1","CODEC_RESTORE_SS_ROT":"1024"},{"CODEC_RESTORE_SS":"1","CODEC_RESTORE_SS_ROT":"2048"},{"CODEC_RESTORE_SS":"1","CODEC_RESTORE_SS_ROT":"4096"},{"CODEC_RESTORE_SS":"1","CODEC_RESTORE_SS_ROT":"263168"},{"CODEC_RESTORE_SS":"1","CODEC_RESTORE_SS_ROT":"2048","CODEC_RESTORE_IL_DEPTH":"16"}]' > gpurun_out/restore_ab.log 2>&1 &&
timeout -k 10 300 python3 -u tools/tune.py --size 512 --rounds 5 --steps 10 --configs '[{},{"CODEC_RESTORE_SS_ROT":"1024"},{"CODEC_RESTORE_SS_ROT":"4096"},{"CODEC_RESTORE_SS_ROT":"17408"}]' > gpurun_out/restore_ab_c3.log 2>&1
