#!/bin/bash
# round-5 N > 1 rehearsals on the box's one GPU (gloo; RCCL needs distinct GPUs), JSON lines with
# the per-rank `ranks` array: 2 ranks at 64 x 2048^2 per rank, 8 ranks at 4 x 512^2 per rank;
# then the default bench again (its traffic_source now names the round-5 PMC summaries)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --batch 64 --steps 5 --warmup 1 --cpu-seconds 0 --c2 0 \
    > gpurun_out/r05/bench_multi2_gloo.json 2> gpurun_out/r05/bench_multi2_gloo.err || { tail -20 gpurun_out/r05/bench_multi2_gloo.err; exit 1; }
echo "multi2 ok"
timeout -k 10 500 python bench.py --gpus 8 --backend gloo --batch 4 --size 512 --steps 2 --warmup 1 --cpu-seconds 0 --c2 0 \
    --payload-chars 256 > gpurun_out/r05/bench_multi8_gloo.json 2> gpurun_out/r05/bench_multi8_gloo.err || { tail -20 gpurun_out/r05/bench_multi8_gloo.err; exit 1; }
echo "multi8 ok"
timeout -k 10 600 python bench.py > gpurun_out/r05/bench.json 2> gpurun_out/r05/bench.err || { tail -20 gpurun_out/r05/bench.err; exit 1; }
echo "bench ok"
