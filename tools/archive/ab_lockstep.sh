#!/bin/bash
# lockstep / early-load A/B over build variants (tools/bin/lib_*.so): restore-path GPU tests
# with the in-tree build, then interleaved bench rounds (LSB + C3 legs)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "restore or c3 or golden or extract" > gpurun_out/ls_tests.log 2>&1; rc=$?
tail -2 gpurun_out/ls_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in tools/bin/lib_base.so tools/bin/lib_se.so tools/bin/lib_sl.so tools/bin/lib_sel.so tools/bin/lib_r3.so tools/bin/lib_res1.so tools/bin/lib_res2.so; do
    timeout -k 10 200 python -u tools/bench_with_lib.py $lib --cpu-seconds 0 --c2 0 --steps 20 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l); c3 = d['c3']
        print(sys.argv[1].split('/')[-1], 'lsb', d['lsb']['ms_per_step'], d['lsb']['kernels_ms'].get('k_scan_rows'),
              '| c3', c3['ms_per_step'], c3['kernels_ms'], '| c3lsb', c3['lsb']['ms_per_step'], c3['lsb']['kernels_ms'], flush=True)
PY
  done
done
