#!/bin/bash
# decision sums: 8 lanes per leaf, branch-free (in-tree) vs the previous library (lib_old.so,
# built from the previous commit's codec_hip.hip); LSB at C3, C2 and the headline shape
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_npsum.txt
: > $OUT
for rep in 1 2 3; do
  for lib in ${LIBS:-default tools/r05/lib_old.so}; do
    echo "== rep $rep lib $lib" >> $OUT
    for args in ${ARGS:-"--size 512" "--size 2048 --batch 1 --steps 20" "--size 2048"}; do
      if [ $lib = default ]; then
        timeout -k 10 200 python tools/tune.py $args --rounds 1 --configs '[{}]' >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
      else
        timeout -k 10 200 python tools/tune_with_lib.py $lib $args --rounds 1 --configs '[{}]' >> $OUT 2>&1 || { tail -5 $OUT; exit 1; }
      fi
    done
  done
done
grep -v amdgpu.ids $OUT
