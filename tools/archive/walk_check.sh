#!/bin/bash
# wide-slice decide check on the GPU box: parity tests that reach k_decide's walk path,
# then the u16 and ct12 LSB steps (walk on / off for u16) and the walk phase stamps
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "wide or kat or batch_vs_oracle or golden" > gpurun_out/walk_tests.log 2>&1
tail -2 gpurun_out/walk_tests.log
for cfg in "u16 1" "u16 0" "ct12 1"; do
  set -- $cfg
  CODEC_DECIDE_WALK=$2 timeout -k 10 200 python -u bench.py --kind $1 --steps 10 --warmup 3 --cpu-seconds 0 --pee 0 --c3 0 \
      > gpurun_out/walk_bench_$1_$2.log 2>&1
  python -c "
import json,sys
for l in open('gpurun_out/walk_bench_$1_$2.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$1 walk=$2', d['ms_per_step'], d.get('kernels_ms'))"
done
timeout -k 10 200 python -u tools/decide_phases_wide.py
