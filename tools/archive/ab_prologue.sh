#!/bin/bash
# ring-first prologues (k_restore_il, k_pee_embed_ss, k_pee_extract_ss, k_pee_embed_res):
# the touched kernels' GPU tests, then an interleaved A/B of two builds over the bench legs
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py \
    -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pro_tests.log 2>&1; rc=$?
tail -2 gpurun_out/pro_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in tools/bin/libold.so tools/bin/libnew.so; do
    timeout -k 10 200 python -u tools/bench_with_lib.py $lib --cpu-seconds 0 --c2 0 --lsb 0 --steps 20 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l)
        ip, c3 = d['inplace'], d['c3']
        print(sys.argv[1].split('/')[-1], 'head', d['ms_per_step'], d['kernels_ms'], '| ip', ip['ms_per_step'], ip['kernels_ms'],
              '| c3', c3['ms_per_step'], c3['kernels_ms'], flush=True)
PY
  done
done
# kernel-argument placement: device-memory kernargs vs the runtime default (latency legs)
for rep in 1 2; do
  for ka in 0 1; do
    HIP_FORCE_DEV_KERNARG=$ka timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 20 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "kernarg=$ka" <<'PY'
import json, sys
for l in open('gpurun_out/ab.log'):
    if l.startswith('{'):
        d = json.loads(l); c2, c3 = d['c2'], d['c3']
        print(sys.argv[1], 'head', d['ms_per_step'], '| c3', c3['ms_per_step'], 'c3lsb', c3['lsb']['ms_per_step'], c3['lsb']['kernels_ms'],
              '| c2 pee', c2['pee']['ms_per_step'], c2['pee']['kernels_ms'], 'c2 lsb', c2['lsb']['ms_per_step'], c2['lsb']['kernels_ms'], flush=True)
PY
  done
done
