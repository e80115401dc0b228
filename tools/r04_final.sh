# round-4 evidence (final tree): GPU suite, smoke, bench, rocprof + PMC (headline), C3 rocprof + PMC,
# C2 rocprof + PMC, then the decision phase stamps at C3 and C2 (diagnostic build)
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/r04_check.sh || exit $?
DTS_B=256 DTS_SIZE=512 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c3_decide_phases.txt 2>&1 || { tail -5 gpurun_out/c3_decide_phases.txt; exit 1; }
DTS_B=1 DTS_SIZE=2048 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c2_decide_phases.txt 2>&1 || { tail -5 gpurun_out/c2_decide_phases.txt; exit 1; }
echo r04-final-done
