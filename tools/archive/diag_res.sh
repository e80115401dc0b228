set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab_res.sh base CODEC_PEE_RES_THREADS=1024 && cat gpurun_out/ab_res.txt && \
timeout -k 10 300 bash tools/res_pmc.sh > gpurun_out/res_pmc.log 2>&1; echo "pmc rc=$?"
