#!/bin/bash
# k_restore_il lockstep A/B (RIL_LOCKSTEP build variants): C3 LSB legs, interleaved
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in tools/bin/libold.so tools/bin/libls1.so tools/bin/libls2.so; do
    timeout -k 10 200 python -u tools/bench_with_lib.py $lib --cpu-seconds 0 --c2 0 --steps 20 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l); c3 = d['c3']
        print(sys.argv[1].split('/')[-1], 'lsb', d['lsb']['ms_per_step'], d['lsb']['kernels_ms'], '| c3lsb', c3['lsb']['ms_per_step'], c3['lsb']['kernels_ms'], flush=True)
PY
  done
done
