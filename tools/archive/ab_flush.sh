#!/bin/bash
# histogram flush bounded by the workgroup's pixel OR: LSB GPU tests, then an interleaved A/B of
# two builds over the LSB legs (headline, C3, C2)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests \
    -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/flush_tests.log 2>&1; rc=$?
tail -2 gpurun_out/flush_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in tools/bin/lib_old.so tools/bin/lib_new.so; do
    timeout -k 10 200 python -u tools/bench_with_lib.py $lib --cpu-seconds 0 --steps 20 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l); c3, c2 = d['c3'], d['c2']
        print(sys.argv[1].split('/')[-1], 'lsb', d['lsb']['ms_per_step'], d['lsb']['kernels_ms'], 'ip', d['lsb']['inplace']['kernels_ms'].get('k_scan_read'),
              '| c3lsb', c3['lsb']['ms_per_step'], c3['lsb']['kernels_ms'], '| c2lsb', c2['lsb']['ms_per_step'], c2['lsb']['kernels_ms'], flush=True)
PY
  done
done
