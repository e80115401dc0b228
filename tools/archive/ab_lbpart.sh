# embed look-back: partial-sum early exit (built in) vs a build without it (tools/bin), headline A/B
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "lookback or headline or kat or flat or small or graph" > gpurun_out/lp_tests.log 2>&1; rc=$?
tail -2 gpurun_out/lp_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python tools/tune_pee.py --batch 256 --size 2048 --modes oop --rounds 3 > gpurun_out/lpA_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/tune_pee.py --lib tools/bin/libcodec_nopart.so --batch 256 --size 2048 --modes oop --rounds 3 > gpurun_out/lpB_$i.log 2>&1 || exit 1
  echo "A (partial exit)"; grep cfg gpurun_out/lpA_$i.log; echo "B (without)"; grep cfg gpurun_out/lpB_$i.log
done
