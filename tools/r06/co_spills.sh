#!/bin/bash
# Spill / scratch report of the LSB kernels in a built library (device code-object notes).
# usage: tools/r06/co_spills.sh LIB.so [NAME_REGEX]
set -euo pipefail
lib=$1; pat=${2:-k_decide|k_scan}
d=$(mktemp -d)
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$d/fb "$lib" /dev/null
$B/clang-offload-bundler --unbundle --type=o --input=$d/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/co
$B/llvm-readelf --notes $d/co | python3 -c '
import re,sys
t=sys.stdin.read(); pat=re.compile(sys.argv[1])
for blk in re.split(r"\n\s+- \.agpr_count", t)[1:]:
    nm=re.search(r"\.name:\s+(\S+)",blk)
    if not nm or not pat.search(nm.group(1)): continue
    g=lambda k: (re.search(r"\."+k+r":\s+(\d+)",blk) or [0,"?"])[1]
    print("%-80s vgpr %4s spill %3s priv %4s" % (nm.group(1)[:80], g("vgpr_count"), g("vgpr_spill_count"), g("private_segment_fixed_size")))
' "$pat"
rm -rf $d
