# inline-hull restore (k_restore_il): restore-path and C3 LSB GPU tests, then an interleaved
# C3 A/B against the copy-then-hull kernel (CODEC_RESTORE_IL=0)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "restore or c3_lsb or golden or extract" > gpurun_out/ril_tests.log 2>&1; rc=$?
tail -2 gpurun_out/ril_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tune.py --batch 256 --size 512 --rounds 5 \
    --configs '[{}, {"CODEC_RESTORE_IL": "0"}]' > gpurun_out/ril_ab.log 2>&1 || exit 1
tail -4 gpurun_out/ril_ab.log
