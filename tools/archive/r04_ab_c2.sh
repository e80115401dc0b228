# round-4 A/B on one box: C2 self-cleaning look-back vs the zeroing launches (MED-PEE 1 x 2048^2),
# in-place slice-serial embed ring (D = 2 refilled late vs D = 1 refilled early), after the PEE
# GPU tests of those paths; then the launch floor
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pee.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "selfclean or graph_replay or matches_oracle or lookback or zeroing or inplace or in_place" > gpurun_out/pytest_sc.log 2>&1 || { tail -30 gpurun_out/pytest_sc.log; exit 1; }
tail -2 gpurun_out/pytest_sc.log
CODEC_PEE_SS_D=1 timeout -k 10 300 python -u -m pytest tests/test_pee.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_ssd1.log 2>&1 || { tail -30 gpurun_out/pytest_ssd1.log; exit 1; }
tail -2 gpurun_out/pytest_ssd1.log
timeout -k 10 300 python tools/tune_pee.py --batch 1 --modes oop --rounds 11 \
  --configs '[{}, {"CODEC_PEE_SELFCLEAN": "0"}]' > gpurun_out/c2_pee_selfclean_ab.log 2>&1 || { tail gpurun_out/c2_pee_selfclean_ab.log; exit 1; }
grep cfg gpurun_out/c2_pee_selfclean_ab.log
timeout -k 10 300 python tools/tune_pee.py --batch 256 --modes ip --rounds 7 \
  --configs '[{}, {"CODEC_PEE_SS_D": "1"}]' > gpurun_out/ip_early_ab.log 2>&1 || { tail gpurun_out/ip_early_ab.log; exit 1; }
grep cfg gpurun_out/ip_early_ab.log
timeout -k 10 120 python tools/launch_floor.py > gpurun_out/launch_floor.json 2>gpurun_out/launch_floor.err || exit 1
cat gpurun_out/launch_floor.json
