#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per pass) over the C2 legs
# (tools/c2_both.py) -> gpurun_out/pmc2_FETCH_SIZE, gpurun_out/pmc2_WRITE_SIZE, plus a
# kernel-trace --stats pass -> gpurun_out/c2prof
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv \
      -d $R/gpurun_out/c2pmc_$C -o run -- python3 $R/tools/c2_both.py 10 > $R/gpurun_out/c2pmc_$C.log 2>&1 ) || exit 1
  tail -1 $R/gpurun_out/c2pmc_$C.log
  mv $R/gpurun_out/c2pmc_$C $R/gpurun_out/pmc2_$C
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/c2prof -o run -- python3 $R/tools/c2_both.py 50 > $R/gpurun_out/c2prof.log 2>&1 ) || exit 1
tail -1 $R/gpurun_out/c2prof.log
