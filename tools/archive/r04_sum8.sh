# 8-lanes-per-leaf wave sums in the decision (np_sum_wave8): LSB parity suites, then C3 / C2 LSB A/B
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sum8.log 2>&1 || { tail -40 gpurun_out/pytest_sum8.log; exit 1; }
tail -2 gpurun_out/pytest_sum8.log
timeout -k 10 300 python tools/tune.py --batch 256 --size 512 --rounds 7 --steps 10 --configs \
  '[{}, {"CODEC_DECIDE_SUM8": "0"}]' > gpurun_out/c3_sum8_ab.log 2>&1 || { tail gpurun_out/c3_sum8_ab.log; exit 1; }
grep cfg gpurun_out/c3_sum8_ab.log
timeout -k 10 200 python tools/tune.py --batch 1 --size 2048 --rounds 9 --steps 10 --configs \
  '[{}, {"CODEC_DECIDE_SUM8": "0"}]' > gpurun_out/c2_sum8_ab.log 2>&1 || { tail gpurun_out/c2_sum8_ab.log; exit 1; }
grep cfg gpurun_out/c2_sum8_ab.log
DTS_B=256 DTS_SIZE=512 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c3_decide_phases.txt 2>&1 || { tail -5 gpurun_out/c3_decide_phases.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/c3_decide_phases.txt
CODEC_DECIDE_SUM8=0 DTS_B=256 DTS_SIZE=512 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c3_decide_phases_old.txt 2>&1 || { tail -5 gpurun_out/c3_decide_phases_old.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/c3_decide_phases_old.txt
