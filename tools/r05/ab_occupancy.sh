#!/bin/bash
# needs the variant libraries first:
#   bash tools/r05/build_variant.sh tools/r05/lib_w45.so -DPEE_E1_WAVES=4 -DPEE_X1_WAVES=5  (and lib_e4 / lib_x5)
# occupancy A/B of the headline look-back passes: the in-tree library against variants built by
# build_variant.sh with __launch_bounds__ minimum waves per SIMD (k_pee_embed1 4: 145 -> 128
# VGPRs; k_pee_extract1 5: 107 -> 95), alternating processes on one box (tools/tune_pee.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
OUT=gpurun_out/r05/ab_occupancy.txt
: > $OUT
for rep in 1 2 3; do
  for lib in default tools/r05/lib_w45.so tools/r05/lib_e4.so tools/r05/lib_x5.so; do
    if [ $lib = default ]; then L=""; else L="--lib $lib"; fi
    echo "== rep $rep lib $lib" >> $OUT
    timeout -k 10 200 python tools/tune_pee.py $L --modes oop --rounds 2 >> $OUT 2>&1 || { echo "failed: $lib"; tail -5 $OUT; exit 1; }
  done
done
cat $OUT | grep -v amdgpu.ids
