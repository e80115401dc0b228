# embed1 finished-flag recheck: PEE GPU tests, then an interleaved headline A/B
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "lookback or headline or kat or flat or small or graph" > gpurun_out/rc_tests.log 2>&1; rc=$?
tail -2 gpurun_out/rc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/tune_pee.py --batch 256 --size 2048 --modes oop --rounds 5 \
    --configs '[{}, {"CODEC_PEE_1P_RECHECK": "0"}]' > gpurun_out/rc_ab.log 2>&1 || exit 1
grep cfg gpurun_out/rc_ab.log
