# C2 MED-PEE latency diagnosis: kernel durations and launch gaps (rocprofv3 kernel trace),
# then the look-back embed's per-slot phase stamps (diagnostic build, tools/lb_trace.py)
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/c2_prof.sh > gpurun_out/c2_gaps.txt 2>&1 || exit 1
cat gpurun_out/c2_gaps.txt
timeout -k 10 120 python tools/lb_trace.py run 1 2>&1 | grep -v amdgpu.ids
