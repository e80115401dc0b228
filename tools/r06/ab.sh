#!/bin/bash
# alternating A/B of two library builds (process per run, 3 reps) on the LSB legs:
#   bash tools/r06/ab.sh tools/r06/lib/lib_prev.so [out name]
set -o pipefail
export CODEC_TUNING=1
OTHER=$1; NAME=${2:-ab}
OUT=gpurun_out/r06/$NAME.txt
mkdir -p gpurun_out/r06; : > $OUT
for rep in 1 2 3; do
  for lib in codec_tcc_amd/libcodec_hip.so $OTHER; do
    for shape in "256 512" "256 2048" "1 2048"; do
      set -- $shape
      echo "== rep $rep lib $lib B=$1 size=$2" >> $OUT
      timeout -k 10 120 python tools/tune_with_lib.py $lib --batch $1 --size $2 --rounds 3 --configs '[{}]' 2>&1 | grep -v amdgpu.ids >> $OUT || exit $?
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, collections
cur = None; res = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith("=="):
        p = l.split(); cur = (p[4], p[5], p[6])
    elif l.startswith("{"):
        d = json.loads(l)
        for k, v in d["kernels_ms"].items(): res[cur + (k,)].append(v)
for k in sorted(res): print(k, [round(x, 4) for x in res[k]])
PY
