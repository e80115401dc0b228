#!/bin/bash
# build libcodec_hip.so from the sources of a git revision (default HEAD) into OUT, for A/B
# against the working tree:  bash tools/r05/build_head.sh tools/r05/lib_old.so [REV]
set -e
cd "$(dirname "$0")/../.."
OUT=$1; REV=${2:-HEAD}
SRC=$(mktemp -d); OBJ=$(mktemp -d)
for f in codec_common.h codec_hip.hip codec_pee.hip codec_quality.hip codec_records.hip; do
  git show "$REV:codec_tcc_amd/csrc/$f" > "$SRC/$f"
done
git show "$REV:include/codec_tcc.h" > "$SRC/codec_tcc.h"
FLAGS="-O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function"
for s in codec_hip codec_pee codec_quality codec_records; do
  /opt/rocm/bin/hipcc $FLAGS -I"$SRC" -c "$SRC/$s.hip" -o "$OBJ/$s.o" 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc $FLAGS -shared "$OBJ"/*.o -o "$OUT"
rm -rf "$SRC" "$OBJ"
echo "built $OUT from $REV"
