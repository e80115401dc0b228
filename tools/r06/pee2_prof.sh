#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/pee2prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/pee2prof -o run -- python3 tools/r06/pee2_prof.py > gpurun_out/r06/pee2prof/out.txt 2>&1; rc=$?
echo "rc $rc"; tail -2 gpurun_out/r06/pee2prof/out.txt
find gpurun_out/r06/pee2prof -name "*kernel_trace.csv" | head -3
exit $rc
