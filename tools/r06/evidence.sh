#!/bin/bash
# round-6 evidence (profiles/r06/): stage "check" = GPU suite, smoke, default bench (CPU
# baselines included); stage "prof" = rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE PMC
# passes of the headline legs, the C3 legs and the C2 legs, and the fast-decision phase
# stamps.  Every step has its own time limit; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 9
R=$GRAFT_REPO_ROOT
STAGE=${1:-check}
mkdir -p gpurun_out/r06
if [ "$STAGE" = check ]; then
  bash tools/gpu_check.sh tests smoke bench || exit $?
fi
if [ "$STAGE" = prof ]; then
  bash tools/gpu_check.sh prof pmc || exit $?
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/c3prof" -o run -- python3 "$R/tools/c3_both.py" 20 > "$R/gpurun_out/c3prof.log" 2>&1 ) || exit 1
  bash tools/c3_pmc.sh || exit 1
  bash tools/c2_pmc.sh || exit 1
  : > gpurun_out/r06/fast_phases.txt
  bash tools/r06/fast_phases.sh || exit 1
fi
echo "r06-$STAGE-done"
