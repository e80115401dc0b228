# round-4 diagnostics: decide phase stamps (C2 split decision, C3 fused), in-place slice-serial trace
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
DTS_B=1 DTS_SIZE=2048 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c2_decide_phases.txt 2>&1 || { tail -5 gpurun_out/c2_decide_phases.txt; exit 1; }
cat gpurun_out/c2_decide_phases.txt | grep -v amdgpu.ids
DTS_B=256 DTS_SIZE=512 timeout -k 10 200 python tools/decide_phases.py ct12 > gpurun_out/c3_decide_phases.txt 2>&1 || { tail -5 gpurun_out/c3_decide_phases.txt; exit 1; }
cat gpurun_out/c3_decide_phases.txt | grep -v amdgpu.ids
timeout -k 10 200 python tools/ss_trace.py run inplace > gpurun_out/ss_trace_inplace.txt 2>&1 || { tail -5 gpurun_out/ss_trace_inplace.txt; exit 1; }
cat gpurun_out/ss_trace_inplace.txt | grep -v amdgpu.ids

timeout -k 10 120 ./tools/bin/ubench_inplace > gpurun_out/ubench_inplace.txt 2>&1 || { tail -5 gpurun_out/ubench_inplace.txt; exit 1; }
cat gpurun_out/ubench_inplace.txt
echo ubench-done
