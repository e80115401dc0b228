# A/B of the pairs' 16-B index loads (np_leaf_list): the LSB parity suites with the new
# library, then C3 and the headline LSB against the previous library, alternating processes
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_leaf16.log 2>&1 || { tail -40 gpurun_out/pytest_leaf16.log; exit 1; }
tail -2 gpurun_out/pytest_leaf16.log
for r in 1 2 3; do
  for L in new prev; do
    timeout -k 10 200 python tools/tune_with_lib.py tools/bin/libcodec_$L.so --batch 256 --size 512 --rounds 3 --steps 10 --configs "[{}]" \
      > gpurun_out/leaf16_c3_$L.$r.log 2>&1 || { tail gpurun_out/leaf16_c3_$L.$r.log; exit 1; }
    echo "c3 $L: $(grep cfg gpurun_out/leaf16_c3_$L.$r.log)"
  done
done
for L in new prev new prev; do
  timeout -k 10 200 python tools/tune_with_lib.py tools/bin/libcodec_$L.so --batch 256 --size 2048 --rounds 2 --steps 5 --configs "[{}]" \
    > gpurun_out/leaf16_hl_$L.log 2>&1 || { tail gpurun_out/leaf16_hl_$L.log; exit 1; }
  echo "headline $L: $(grep cfg gpurun_out/leaf16_hl_$L.log)"
done
