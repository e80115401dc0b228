#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=8 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -45 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; brc=$?
  echo "bench rc=$brc"; cat gpurun_out/bench.json; tail -20 gpurun_out/bench.err
fi
