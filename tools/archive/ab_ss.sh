#!/bin/bash
# headline PEE step: slice-serial forced (CODEC_PEE_SS=1) vs the default dispatch, interleaved
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for i in 1 2 3; do for v in 1 -1; do
  CODEC_PEE_SS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --lsb 0 --c2 0 --c3 0 --cpu-seconds 0 \
      > gpurun_out/ss_$v.json 2> gpurun_out/ss_$v.err || { tail -5 gpurun_out/ss_$v.err; exit 1; }
  echo "SS=$v"; python tools/bench_brief.py gpurun_out/ss_$v.json | head -2
done; done
