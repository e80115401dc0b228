#!/bin/bash
# A/B of two library builds on one box: bash tools/ab_libs.sh LIB_A LIB_B [bench args...]
# prints ms_per_step and the decide kernel time of each, twice, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for rep in 1 2; do
  for lib in $A $B; do
    timeout -k 10 200 python -u tools/bench_with_lib.py $lib "$@" > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l); k = d['kernels_ms']
        print(sys.argv[1].split('/')[-1], d['ms_per_step'], {n: v for n, v in k.items() if 'decide' in n},
              'c3', (d.get('c3') or {}).get('ms_per_step'))
PY
  done
done
