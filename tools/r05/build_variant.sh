#!/bin/bash
# build a variant of libcodec_hip.so with extra -D flags (A/B of build-time knobs on one box):
#   bash tools/r05/build_variant.sh OUT.so -DPEE_E1_WAVES=4 -DPEE_X1_WAVES=5
set -e
cd "$(dirname "$0")/../.."
OUT=$1; shift
TMP=$(mktemp -d)
FLAGS="-O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
for s in codec_hip codec_pee codec_quality codec_records; do
  /opt/rocm/bin/hipcc $FLAGS -Iinclude -c codec_tcc_amd/csrc/$s.hip -o $TMP/$s.o &
done
wait
/opt/rocm/bin/hipcc $FLAGS -shared $TMP/*.o -o "$OUT"
rm -rf "$TMP"
echo "built $OUT ($*)"
