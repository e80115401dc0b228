# slice-serial extract: ring refilled early (in place by default now: depth 1) -- the PEE suite with
# the defaults and with the out-of-place early variant forced, then in-place and C3 A/B
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pee.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_xearly.log 2>&1 || { tail -30 gpurun_out/pytest_xearly.log; exit 1; }
echo "defaults: $(tail -1 gpurun_out/pytest_xearly.log)"
CODEC_PEE_SSX_EARLY=1 CODEC_PEE_SSX_D=1 timeout -k 10 300 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_xearly_oop.log 2>&1 || { tail -30 gpurun_out/pytest_xearly_oop.log; exit 1; }
echo "early everywhere: $(tail -1 gpurun_out/pytest_xearly_oop.log)"
timeout -k 10 300 python tools/tune_pee.py --batch 256 --modes ip --rounds 7 --configs \
  '[{}, {"CODEC_PEE_SSX_EARLY": "0"}]' > gpurun_out/ip_xearly_ab2.log 2>&1 || { tail gpurun_out/ip_xearly_ab2.log; exit 1; }
grep cfg gpurun_out/ip_xearly_ab2.log
timeout -k 10 300 python tools/tune_pee.py --batch 256 --size 512 --T auto --modes oop --rounds 7 --configs \
  '[{}, {"CODEC_PEE_SSX_EARLY": "1", "CODEC_PEE_SSX_D": "1"}, {"CODEC_PEE_SSX_EARLY": "1", "CODEC_PEE_SSX_D": "2"}]' \
  > gpurun_out/c3_xearly_ab.log 2>&1 || { tail gpurun_out/c3_xearly_ab.log; exit 1; }
grep cfg gpurun_out/c3_xearly_ab.log
