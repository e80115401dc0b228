#!/bin/bash
# C2 MED-PEE kernel times, library A (argument) against the in-tree build B, interleaved:
#   bash tools/c2_ab.sh tools/bin/libcodec_old.so [rounds]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="$1"; N="${2:-2}"
for i in $(seq 1 "$N"); do
  for v in A B; do
    if [ "$v" = A ]; then lib="$R/$A"; else lib=""; fi
    CODEC_TCC_LIB="$lib" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c2$v -o run \
        -- python3 $R/tools/c2_pee.py 200 > $R/gpurun_out/c2$v.log 2>&1 || exit 1
    echo "== $v $i $(tail -1 $R/gpurun_out/c2$v.log)"
    (cd $R && python tools/rocprof_summary.py gpurun_out/c2$v/run_kernel_trace.csv x 5 | grep -E "k_|fillBuffer|copyBuffer")
  done
done
