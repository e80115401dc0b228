# per-wave end stamps of the decision's first MI round at C3 (diagnostic build)
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
DTS_B=256 DTS_SIZE=512 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c3_decide_waves.txt 2>&1 || { tail -5 gpurun_out/c3_decide_waves.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/c3_decide_waves.txt
