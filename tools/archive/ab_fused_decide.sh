# fused scan + decide (k_scan_decide): LSB GPU parity tests (golden cases through every decision
# path incl. the fused one), C3 LSB config test, then the C3 A/B against the separate kernels
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "not headline" > gpurun_out/fd_tests.log 2>&1; rc=$?
tail -15 gpurun_out/fd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tune.py --batch 256 --size 512 --rounds 5 \
    --configs '[{}, {"CODEC_FUSED_DECIDE": "0"}]' > gpurun_out/fd_ab.log 2>&1 || exit 1
grep cfg gpurun_out/fd_ab.log
