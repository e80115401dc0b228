#!/bin/bash
# A/B of two builds of the library on the GPU box, interleaved rounds of the PEE legs:
#   bash tools/ab_bench.sh tools/bin/libcodec_old.so [rounds] [extra bench args]
# B = the in-tree codec_tcc_amd/libcodec_hip.so.  Writes gpurun_out/ab_{A,B}_<i>.json.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
A="$1"; N="${2:-3}"; shift 2
for i in $(seq 1 "$N"); do
  for v in A B; do
    if [ "$v" = A ]; then lib="$A"; else lib=""; fi
    CODEC_TCC_LIB="$lib" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --lsb 0 --c2 0 --cpu-seconds 0 "$@" \
        > "gpurun_out/ab_${v}_$i.json" 2> "gpurun_out/ab_${v}_$i.err" || { echo "bench $v $i failed"; tail -5 "gpurun_out/ab_${v}_$i.err"; exit 1; }
    python - "$v" "gpurun_out/ab_${v}_$i.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ip, c3 = d.get("inplace", {}), d.get("c3", {})
print(sys.argv[1], "step", d["ms_per_step"], d.get("kernels_ms"), "| inplace", ip.get("ms_per_step"), ip.get("kernels_ms"),
      "| c3", c3.get("ms_per_step"), c3.get("kernels_ms"), "| ok", d["roundtrip_ok"], ip.get("roundtrip_ok"), c3.get("roundtrip_ok"))
EOF
  done
done
