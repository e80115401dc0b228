# A/B of k_pee_embed_res launch variants at C3 (phase timeline of tools/res_trace.py per variant)
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  env CODEC_PEE_RES_TRACE=1 $e timeout -k 10 200 python tools/res_trace.py > gpurun_out/rt.txt 2>&1 || exit 1
  echo "== $v" >> gpurun_out/ab_res.txt; grep -v amdgpu gpurun_out/rt.txt >> gpurun_out/ab_res.txt
done
