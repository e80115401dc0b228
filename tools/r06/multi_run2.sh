#!/bin/bash
# MED-PEE GPU suite, then the default bench line (C3 carries pee_scheme2)
set -o pipefail
bash tools/r06/multi_run.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r06/bench_multi.json 2> gpurun_out/r06/bench_multi.err; rc=$?
echo "bench rc $rc"
exit $rc
