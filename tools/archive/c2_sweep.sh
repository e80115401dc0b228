#!/bin/bash
# C2 MED-PEE kernel times under a few launch knobs (rocprofv3 kernel trace)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "X=1" "CODEC_NT=0" "CODEC_PEE_ONEPASS=0" "CODEC_PEE_FLAT_MAXB=0" "CODEC_PEE_FLAT_TICKET=1" "CODEC_PEE_LB_SPINS=64"; do
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c2 -o run -- python3 $R/tools/c2_pee.py 50 > $R/gpurun_out/c2.log 2>&1 || exit 1
  echo "== $cfg $(tail -1 $R/gpurun_out/c2.log)"; (cd $R && python tools/rocprof_summary.py gpurun_out/c2/run_kernel_trace.csv x 5 | grep -E "k_|fillBuffer|copyBuffer")
done
