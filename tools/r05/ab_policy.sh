#!/bin/bash
export CODEC_TUNING=1   # CODEC_* knobs are honoured only under the tuning switch
# cache-policy A/B: the in-tree library (non-temporal vector loads and stores where the kernels
# ask for them) against builds with plain stores / plain loads, alternating processes on one box
#   bash tools/r05/build_variant.sh tools/r05/lib_pst.so -DCODEC_PLAIN_STORES=1
#   bash tools/r05/build_variant.sh tools/r05/lib_pld.so -DCODEC_PLAIN_LOADS=1
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_policy.txt
: > $OUT
for rep in 1 2 3; do
  for lib in default tools/r05/lib_pst.so tools/r05/lib_pld.so; do
    if [ $lib = default ]; then L=""; LL=""; else L="--lib $lib"; LL="$lib"; fi
    echo "== rep $rep lib $lib" >> $OUT
    timeout -k 10 200 python tools/tune_pee.py $L --modes oop,ip --rounds 1 >> $OUT 2>&1 || { echo "failed pee: $lib"; tail -5 $OUT; exit 1; }
    if [ -z "$LL" ]; then
      timeout -k 10 200 python tools/tune.py --rounds 1 --configs '[{}]' >> $OUT 2>&1 || { echo "failed lsb"; tail -5 $OUT; exit 1; }
    else
      timeout -k 10 200 python tools/tune_with_lib.py $LL --rounds 1 --configs '[{}]' >> $OUT 2>&1 || { echo "failed lsb: $lib"; tail -5 $OUT; exit 1; }
    fi
  done
done
grep -v amdgpu.ids $OUT
