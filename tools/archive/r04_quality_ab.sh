# A/B of k_quality's accumulators (32-bit sums + float64 FMAs vs 64-bit multiply-adds): the
# quality GPU tests with the new library, then the headline-size k_quality against the previous
# library, alternating processes
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_quality.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_quality.log 2>&1 || { tail -30 gpurun_out/pytest_quality.log; exit 1; }
tail -1 gpurun_out/pytest_quality.log
for r in 1 2 3; do
  for L in new prev; do
    timeout -k 10 200 python tools/quality_time.py tools/bin/libcodec_$L.so > gpurun_out/q_$L.$r.log 2>&1 || { tail gpurun_out/q_$L.$r.log; exit 1; }
    echo "$L: $(tail -1 gpurun_out/q_$L.$r.log)"
  done
done
