#!/bin/bash
# build the library of a git revision (its csrc/ + include/) into OUT.so for A/B runs:
#   bash tools/r06/build_rev.sh HEAD tools/r06/lib/lib_prev.so [-DEXTRA ...]
set -e
cd "$(dirname "$0")/../.."
REV=$1; OUT=$(realpath -m "$2"); shift 2
TMP=$(mktemp -d)
mkdir -p $TMP/codec_tcc_amd/csrc $TMP/include
for f in codec_hip.hip codec_pee.hip codec_quality.hip codec_records.hip codec_common.h; do
  git show "$REV:codec_tcc_amd/csrc/$f" > $TMP/codec_tcc_amd/csrc/$f
done
git show "$REV:include/codec_tcc.h" > $TMP/include/codec_tcc.h
FLAGS="-O3 -std=c++17 -ffp-contract=off -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
for s in codec_hip codec_pee codec_quality codec_records; do
  /opt/rocm/bin/hipcc $FLAGS -I$TMP/include -c $TMP/codec_tcc_amd/csrc/$s.hip -o $TMP/$s.o &
done
wait
/opt/rocm/bin/hipcc $FLAGS -shared $TMP/*.o -o "$OUT"
rm -rf "$TMP"
echo "built $OUT from $REV"
