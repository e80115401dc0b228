#!/bin/bash
# GPU box check: build, pytest -m gpu, bench, rocprofv3 kernel stats (+ optional PMC passes).
# usage: bash tools/gpu_check.sh [tests] [bench] [prof] [pmc]   (default: tests bench prof)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
STAGES="${*:-tests bench prof}"
has() { [[ " $STAGES " == *" $1 "* ]]; }
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
  [ $rc -le 1 ] || exit $rc
fi
if has smoke; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  R="$GRAFT_REPO_ROOT"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --c3 0 --c2 0 \
      > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.log" ); rc=$?
  echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
  [ $rc -eq 0 ] || exit $rc
fi
if has multi; then
  # 2-rank rehearsal of the N>1 path on this 1-GPU box (gloo: RCCL needs distinct GPUs)
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --batch 64 --backend gloo --cpu-seconds 0 \
      > gpurun_out/bench_multi.json 2> gpurun_out/bench_multi.err; rc=$?
  echo "multi rc=$rc"; cat gpurun_out/bench_multi.json; tail -5 gpurun_out/bench_multi.err
  [ $rc -eq 0 ] || exit $rc
fi
if has pmc; then
  R="$GRAFT_REPO_ROOT"
  for C in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv \
        -d "$R/gpurun_out/pmc_$C" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-profile --c3 0 --c2 0 \
        > "$R/gpurun_out/pmc_$C.log" 2>&1 ); rc=$?
    echo "pmc $C rc=$rc"; tail -2 "gpurun_out/pmc_$C.log"
    [ $rc -eq 0 ] || exit $rc
  done
fi
