#!/bin/bash
# k_pee_embed_res build variants (RES_LOCKSTEP / RES_ELOCK / RES_G1024): C3 PEE legs, interleaved
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in tools/bin/lib_base.so tools/bin/lib_g1.so tools/bin/lib_g3.so tools/bin/lib_g4.so; do
    timeout -k 10 200 python -u tools/bench_with_lib.py $lib --cpu-seconds 0 --c2 0 --lsb 0 --steps 20 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l); c3 = d['c3']
        print(sys.argv[1].split('/')[-1], '| c3', c3['ms_per_step'], c3['kernels_ms'], flush=True)
PY
  done
done
