cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/tune_pee.py --lib tools/bin/libcodec_fused1.so --batch 256 --size 512 --T auto --rounds 3 > gpurun_out/abA_$i.log 2>&1 || exit 1
  timeout -k 10 200 python tools/tune_pee.py --batch 256 --size 512 --T auto --rounds 3 > gpurun_out/abB_$i.log 2>&1 || exit 1
  echo A; cat gpurun_out/abA_$i.log | grep cfg; echo B; cat gpurun_out/abB_$i.log | grep cfg
done
