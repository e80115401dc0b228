#!/bin/bash
# LSB step kernel times under launch knobs:  bash tools/lsb_sweep.sh <BxHxW> "<cfg>" "<cfg>" ...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
shape="$1"; shift
for cfg in "$@"; do
  env LSB_SHAPE=$shape $cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lsw -o run -- python3 $R/tools/c3_lsb.py 30 > $R/gpurun_out/lsw.log 2>&1 || exit 1
  echo "== $shape $cfg $(tail -1 $R/gpurun_out/lsw.log)"; (cd $R && python tools/rocprof_summary.py gpurun_out/lsw/run_kernel_trace.csv x 5 | grep -E "k_|fill|copy")
done
