#!/bin/bash
export CODEC_TUNING=1   # CODEC_* knobs are honoured only under the tuning switch
# wave scan by DPP (in-tree) vs ds_bpermute shuffles (lib_old.so: -DCODEC_WSCAN_DPP=0):
# MED-PEE headline and C3 (tune_pee.py), LSB at C3 / C2 / headline (tune.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_wscan.txt
: > $OUT
for rep in 1 2 3; do
  for lib in default tools/r05/lib_old.so; do
    if [ $lib = default ]; then L=""; else L="--lib $lib"; fi
    echo "== rep $rep lib $lib" >> $OUT
    timeout -k 10 200 python tools/tune_pee.py $L --modes oop,ip --rounds 1 >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
    timeout -k 10 200 python tools/tune_pee.py $L --size 512 --T auto --modes oop --rounds 1 >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
    for args in "--size 512" "--size 2048 --batch 1 --steps 20" "--size 2048"; do
      if [ $lib = default ]; then
        timeout -k 10 200 python tools/tune.py $args --rounds 1 --configs '[{}]' >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
      else
        timeout -k 10 200 python tools/tune_with_lib.py $lib $args --rounds 1 --configs '[{}]' >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
      fi
    done
  done
done
grep -v amdgpu.ids $OUT
