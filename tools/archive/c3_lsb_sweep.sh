cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "X=1" "CODEC_RESTORE_GS_THREADS=256" "CODEC_FUSED_GATHER=0" "CODEC_RESTORE_GS_WGS=1024"; do
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c3l -o run -- python3 $R/tools/c3_lsb.py 20 > $R/gpurun_out/c3l.log 2>&1 || exit 1
  echo "== $cfg"; (cd $R && python tools/rocprof_summary.py gpurun_out/c3l/run_kernel_trace.csv x | grep "k_" )
done
