#!/usr/bin/env python3
"""Per-kernel instruction mix from a device assembly file (hipcc --cuda-device-only -S):
    python tools/isa_stats.py pee.s k_pee_embed_ss [substring of the mangled name ...]
Prints, for each matching kernel, the instruction count per class, the VGPR/SGPR/LDS usage
and the basic blocks with their sizes (to find the per-chunk loop body)."""
import collections
import re
import sys

path, pats = sys.argv[1], sys.argv[2:]
lines = open(path).read().split("\n")
starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w+:\s*(;.*)?$", l)]
for si, s in enumerate(starts):
    name = lines[s].split(":")[0]
    if not all(p in name for p in pats):
        continue
    end = next((j for j in range(s, len(lines)) if lines[j].strip().startswith(".Lfunc_end")), len(lines))
    body = lines[s:end]
    mix = collections.Counter()
    blocks = []
    cur = [name, 0]
    for l in body:
        t = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", t):
            blocks.append(cur)
            cur = [t.split(":")[0], 0]
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cur[1] += 1
        cls = op.split("_")[0]
        if op.startswith("s_waitcnt") or op.startswith("s_barrier"):
            cls = op
        mix[cls] += 1
    blocks.append(cur)
    meta = {}
    for j in range(end, min(end + 60, len(lines))):
        m = re.match(r"\s*;\s*(NumVgprs|NumSgprs|ScratchSize|Occupancy|LDSByteSize|NumAgprs|TotalNumVgprs):\s*(\d+)", lines[j])
        if m:
            meta[m.group(1)] = int(m.group(2))
    print(name)
    print("  ", meta)
    print("  ", dict(mix.most_common()))
    print("   blocks:", ", ".join(f"{b}:{n}" for b, n in blocks if n))
