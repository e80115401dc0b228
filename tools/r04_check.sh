# round-4 evidence: GPU suite, smoke, bench, rocprof + PMC (headline), C3 rocprof + PMC, C2 rocprof + PMC
cd "$GRAFT_REPO_ROOT" || exit 9
R=$GRAFT_REPO_ROOT
bash tools/gpu_check.sh tests smoke bench prof pmc || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/c3prof" -o run -- python3 "$R/tools/c3_both.py" 20 > "$R/gpurun_out/c3prof.log" 2>&1 ) || exit 1
bash tools/c3_pmc.sh || exit 1
bash tools/c2_pmc.sh || exit 1
echo r04-check-done
