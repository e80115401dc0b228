#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per pass) over the C3 legs
# (tools/c3_both.py) -> gpurun_out/c3pmc_FETCH_SIZE, gpurun_out/c3pmc_WRITE_SIZE
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv \
      -d $R/gpurun_out/c3pmc_$C -o run -- python3 $R/tools/c3_both.py 5 > $R/gpurun_out/c3pmc_$C.log 2>&1 ) || exit 1
  tail -1 $R/gpurun_out/c3pmc_$C.log
  mv $R/gpurun_out/c3pmc_$C $R/gpurun_out/pmc3_$C
done
