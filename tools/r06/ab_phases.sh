#!/bin/bash
# LSB suites + A/B against OTHER + fast-decision phase stamps
set -o pipefail
bash tools/r06/ab_run.sh "$@" || exit $?
: > gpurun_out/r06/fast_phases.txt
bash tools/r06/fast_phases.sh
