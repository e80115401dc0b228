#!/bin/bash
# MED-PEE GPU suite (scheme 1 + scheme 2)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_pee.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06/pytest_pee.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "^FAILED|^ERROR" gpurun_out/r06/pytest_pee.log | head -20; tail -1 gpurun_out/r06/pytest_pee.log
exit $rc
