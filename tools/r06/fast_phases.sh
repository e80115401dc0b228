#!/bin/bash
# fast-decision phase stamps at C3, C2 and 64 x 2048^2 (diagnostic library in tools/r06/lib)
set -o pipefail
mkdir -p gpurun_out/r06
export DTS_LIB=tools/r06/lib/libcodec_hip_dts.so
for cfg in "512 256" "2048 1" "2048 64"; do
  set -- $cfg
  DTS_SIZE=$1 DTS_B=$2 timeout -k 10 120 python -u tools/r06/fast_phases.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06/fast_phases.txt || exit $?
done
