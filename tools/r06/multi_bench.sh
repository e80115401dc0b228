#!/bin/bash
# scheme-2 container/pipeline GPU tests, then the default bench line (its C3 leg carries pee_scheme2)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest tests/test_container_dicom.py -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06/pytest_container.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "^FAILED|^ERROR" gpurun_out/r06/pytest_container.log | head; tail -1 gpurun_out/r06/pytest_container.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r06/bench_multi.json 2> gpurun_out/r06/bench_multi.err; rc=$?
echo "bench rc $rc"; tail -3 gpurun_out/r06/bench_multi.err
exit $rc
