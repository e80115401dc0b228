# round-end evidence: full GPU suite, smoke, bench, rocprof (headline + C3), C3 PMC passes
cd "$GRAFT_REPO_ROOT" || exit 9
R=$GRAFT_REPO_ROOT
bash tools/gpu_check.sh tests smoke bench prof || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/c3prof" -o run -- python3 "$R/tools/c3_both.py" 20 > "$R/gpurun_out/c3prof.log" 2>&1 ) || exit 1
bash tools/c3_pmc.sh || exit 1
echo final-check-done
