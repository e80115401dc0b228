#!/bin/bash
# C2 MED-PEE step under rocprofv3 --kernel-trace: per-kernel durations and the gaps between
# consecutive launches (tools/c2_gaps.py)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c2p -o run -- python3 $R/tools/c2_pee.py 200 > $R/gpurun_out/c2p.log 2>&1 || exit 1
cd $R && python tools/rocprof_summary.py gpurun_out/c2p/run_kernel_trace.csv "C2 MED-PEE, 200 steps" 20
cd $GRAFT_REPO_ROOT && python tools/c2_gaps.py gpurun_out/c2p/run_kernel_trace.csv 400
