# round-4 quick GPU check: PEE tests (self-cleaning look-back, graph replay, oracle parity, fallbacks),
# the distributed GPU tests, a bench without CPU baselines, the in-place ubench
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -u -m pytest tests/test_pee.py tests/test_distributed_gpu.py -m gpu -q --maxfail=8 -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_quick.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 --lsb 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err; rc=$?
echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/bench_quick.json').read().strip().splitlines()[-1])
print('head', d['value'], d['ms_per_step'], d['kernels_ms'], d['roundtrip_ok'])
print('inplace', d['inplace']['ms_per_step'], d['inplace']['kernels_ms'], d['inplace']['roundtrip_ok'])
print('c3', d['c3']['ms_per_step'], d['c3']['kernels_ms'], d['c3']['roundtrip_ok'])
print('c2 pee', d['c2']['pee']['ms_per_step'], d['c2']['pee']['kernels_ms'], d['c2']['pee']['roundtrip_ok'])
print('c2 lsb', d['c2']['lsb']['ms_per_step'], d['c2']['lsb']['kernels_ms'], d['c2']['lsb']['roundtrip_ok'])
" || exit 1
timeout -k 10 120 ./tools/bin/ubench_inplace > gpurun_out/ubench_inplace.txt 2>&1 || exit 1
cat gpurun_out/ubench_inplace.txt
echo quick-done
