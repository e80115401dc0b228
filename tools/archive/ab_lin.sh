# LIN resident embed: GPU tests of the fused auto embed, then an interleaved C3 A/B of the
# resident launches (LIN 1024 / cursor 1024 / 512 threads) and the phase trace of the default
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "fused_edges or c3_pee or capacity" > gpurun_out/lin_tests.log 2>&1; rc=$?
tail -3 gpurun_out/lin_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tune_pee.py --batch 256 --size 512 --T auto --modes oop --rounds 5 \
    --configs '[{}, {"CODEC_PEE_RES_LIN": "0"}, {"CODEC_PEE_RES_THREADS": "512"}]' > gpurun_out/lin_ab.log 2>&1 || exit 1
cat gpurun_out/lin_ab.log | grep cfg
CODEC_PEE_RES_TRACE=1 timeout -k 10 200 python tools/res_trace.py 2>&1 | grep -v amdgpu
