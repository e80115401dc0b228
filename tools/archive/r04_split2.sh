# The split decision's plane workgroups with the terms' table loads in flight through the
# list build, and the main workgroup's H(Y) on two waves (CODEC_DECIDE_SPLIT2=0: before):
# LSB parity suites, then C2 LSB with and without, alternating in one process
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_split2.log 2>&1 || { tail -40 gpurun_out/pytest_split2.log; exit 1; }
tail -1 gpurun_out/pytest_split2.log
timeout -k 10 300 python3 -u tools/tune.py --batch 1 --rounds 7 --steps 20 --configs '[{},{"CODEC_DECIDE_SPLIT2":"0"},{},{"CODEC_DECIDE_SPLIT2":"0"}]' 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 -u tools/tune.py --batch 4 --size 1024 --rounds 5 --steps 20 --configs '[{},{"CODEC_DECIDE_SPLIT2":"0"}]' 2>&1 | grep -v amdgpu.ids
