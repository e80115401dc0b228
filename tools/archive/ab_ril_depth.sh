# C3 LSB restore: k_restore_il ring depth A/B (4 / 8 / 16 vectors per thread)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune.py --batch 256 --size 512 --rounds 5 \
    --configs '[{}, {"CODEC_RESTORE_IL_DEPTH": "4"}, {"CODEC_RESTORE_IL_DEPTH": "16"}]' > gpurun_out/ril_depth.log 2>&1 || exit 1
grep cfg gpurun_out/ril_depth.log
