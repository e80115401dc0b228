#!/bin/bash
export CODEC_TUNING=1   # CODEC_* knobs are honoured only under the tuning switch
# write-through (sc1 / sc0 sc1) instead of non-temporal 16-B stores, alternating processes:
#   bash tools/r05/build_variant.sh tools/r05/lib_sc1.so -DCODEC_ST_SC=1
#   bash tools/r05/build_variant.sh tools/r05/lib_sc01.so -DCODEC_ST_SC=3
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_store_sc.txt
: > $OUT
for rep in 1 2 3; do
  for lib in default tools/r05/lib_sc1.so tools/r05/lib_sc01.so; do
    if [ $lib = default ]; then L=""; else L="--lib $lib"; fi
    echo "== rep $rep lib $lib" >> $OUT
    timeout -k 10 200 python tools/tune_pee.py $L --modes oop --rounds 1 >> $OUT 2>&1 || { echo "failed pee: $lib"; tail -5 $OUT; exit 1; }
    timeout -k 10 200 python tools/tune_pee.py $L --size 512 --T auto --modes oop --rounds 1 >> $OUT 2>&1 || { echo "failed c3: $lib"; tail -5 $OUT; exit 1; }
    if [ $lib = default ]; then
      timeout -k 10 200 python tools/tune.py --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
      timeout -k 10 200 python tools/tune.py --size 512 --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
    else
      timeout -k 10 200 python tools/tune_with_lib.py $lib --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
      timeout -k 10 200 python tools/tune_with_lib.py $lib --size 512 --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
    fi
  done
done
grep -v amdgpu.ids $OUT
