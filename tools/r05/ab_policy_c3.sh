#!/bin/bash
# cache-policy A/B at C3 (256 x 512^2: MED-PEE T=auto out of place and in place, LSB) and the
# LSB in-place step at the headline shape; libraries as in ab_policy.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_policy_c3.txt
: > $OUT
for rep in 1 2 3; do
  for lib in default tools/r05/lib_pst.so tools/r05/lib_pld.so; do
    if [ $lib = default ]; then L=""; else L="--lib $lib"; fi
    echo "== rep $rep lib $lib" >> $OUT
    timeout -k 10 200 python tools/tune_pee.py $L --size 512 --T auto --modes oop,ip --rounds 1 >> $OUT 2>&1 || { echo "failed pee: $lib"; tail -5 $OUT; exit 1; }
    if [ $lib = default ]; then
      timeout -k 10 200 python tools/tune.py --size 512 --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
      timeout -k 10 200 python tools/tune.py --inplace --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
    else
      timeout -k 10 200 python tools/tune_with_lib.py $lib --size 512 --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
      timeout -k 10 200 python tools/tune_with_lib.py $lib --inplace --rounds 1 --configs '[{}]' >> $OUT 2>&1 || exit 1
    fi
  done
done
grep -v amdgpu.ids $OUT
