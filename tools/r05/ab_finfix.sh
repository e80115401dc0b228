#!/bin/bash
# headline MED-PEE: the finished-flag fix (in-tree) vs the previous commit's library (lib_old.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_finfix.txt
: > $OUT
for rep in 1 2 3 4; do
  for lib in default tools/r05/lib_old.so; do
    if [ $lib = default ]; then L=""; else L="--lib $lib"; fi
    echo "== rep $rep lib $lib" >> $OUT
    timeout -k 10 200 python tools/tune_pee.py $L --modes oop --rounds 1 >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
  done
done
grep -v amdgpu.ids $OUT
