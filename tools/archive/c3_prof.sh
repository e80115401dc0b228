# C3 evidence run: GPU tests of the fused auto embed, the C3 PEE A/B line, a rocprofv3
# kernel-stats pass over both C3 legs (tools/c3_both.py) and the FETCH_SIZE / WRITE_SIZE passes
cd "$GRAFT_REPO_ROOT" || exit 9
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "fused_edges or c3_pee or capacity" > gpurun_out/c3_tests.log 2>&1; rc=$?
tail -2 gpurun_out/c3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tune_pee.py --batch 256 --size 512 --T auto --modes oop --rounds 5 > gpurun_out/c3_ab.log 2>&1 || exit 1
grep cfg gpurun_out/c3_ab.log
CODEC_PEE_RES_TRACE=1 timeout -k 10 200 python tools/res_trace.py 2>&1 | grep -v amdgpu
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/c3prof" -o run -- python3 "$R/tools/c3_both.py" 20 > "$R/gpurun_out/c3prof.log" 2>&1 ) || exit 1
bash tools/c3_pmc.sh || exit 1
