#!/bin/bash
# tools/tune.py (LSB kernels) under two library builds, alternating:
#   bash tools/ab_tune_libs.sh LIB_A LIB_B [tune.py args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for rep in 1 2; do
  for lib in $A $B; do
    CODEC_TCC_LIB=$lib timeout -k 10 200 python tools/tune.py --configs "[{}]" "$@" > gpurun_out/abt.log 2>&1 || { tail -5 gpurun_out/abt.log; exit 1; }
    echo "$(basename $lib) $(grep cfg gpurun_out/abt.log)"
  done
done
