"""A second, independent statement of the MED-PEE scheme: scalar Python loops written from
the specification in oracle/pee_cpu.py's header (one candidate at a time, no numpy
vectorisation).  Test infrastructure: it cross-checks the vectorised oracle on small images
and generates the scheme's known-answer vectors (tests/golden/make_pee_golden.py), which
freeze the definition that the version-16 STGC container's files depend on.  The reference
repository has no PEE code, so neither this nor the oracle is pinned to it (parity unpinned).
"""
from __future__ import annotations


def _med(a: int, b: int, c: int) -> int:
    if c >= max(a, b):
        return min(a, b)
    if c <= min(a, b):
        return max(a, b)
    return a + b - c


# scheme 2's sublattices as (row parity, column parity); 0 is scheme 1's (odd, odd)
LATTICES = ((1, 1), (0, 0), (1, 0), (0, 1))


def _cands(img, lattice=0):
    """(k, y, x, value, prediction) of every candidate in index order: pixels whose row and
    column parities are the lattice's, with y >= 1 and x >= 1, row by row."""
    H, W = len(img), len(img[0])
    ry, rx = LATTICES[lattice]
    out = []
    for y in range(1, H):
        if y % 2 != ry:
            continue
        for x in range(1, W):
            if x % 2 != rx:
                continue
            p = _med(img[y][x - 1], img[y - 1][x], img[y - 1][x - 1])
            out.append((len(out), y, x, img[y][x], p))
    return out


def embed(img, bits, T: int, maxval: int, truncate: bool = True, lattice: int = 0):
    """img: list of lists of ints -> (stego rows, side dict) as pee_cpu.pee_embed."""
    cands = _cands(img, lattice)
    kinds = []
    for _k, _y, _x, v, p in cands:
        e = v - p
        if -T <= e < T:
            kinds.append(("e", 0 <= p + 2 * e and p + 2 * e + 1 <= maxval))
        elif e >= T:
            kinds.append(("r", v + T <= maxval))
        else:
            kinds.append(("l", v - T >= 0))
    capacity = sum(1 for kd, ok in kinds if kd == "e" and ok)
    L, status = len(bits), 0
    if capacity < L:
        if not truncate:
            raise ValueError("payload exceeds the capacity")
        bits, L, status = bits[:capacity], capacity, 1
        end = len(cands) - 1
    else:
        end, seen = -1, 0
        for idx, (kd, ok) in enumerate(kinds):
            if L and kd == "e" and ok:
                seen += 1
                if seen == L:
                    end = idx
                    break
    out = [list(r) for r in img]
    lm = []
    cur = 0
    for idx, ((_k, y, x, v, p), (kd, ok)) in enumerate(zip(cands, kinds)):
        if idx > end:
            break
        lm.append(not ok)
        if not ok:
            continue
        if kd == "e":
            out[y][x] = p + 2 * (v - p) + int(bits[cur])
            cur += 1
        elif kd == "r":
            out[y][x] = v + T
        else:
            out[y][x] = v - T
    return out, {"T": T, "L": L, "end": end, "lm": lm, "capacity": capacity, "status": status, "lattice": lattice}


def extract(stego, side):
    T, end, L = side["T"], side["end"], side["L"]
    out = [list(r) for r in stego]
    bits = []
    for idx, (_k, y, x, v, p) in enumerate(_cands(stego, side.get("lattice", 0))):
        if idx > end:
            break
        if side["lm"][idx]:
            continue
        e2 = v - p
        if -2 * T <= e2 < 2 * T:
            bits.append(e2 & 1)
            out[y][x] = p + (e2 >> 1)
        elif e2 >= 2 * T:
            out[y][x] = v - T
        else:
            out[y][x] = v + T
    return bits[:L], out


def embed_multi(img, bits, T: int, maxval: int, passes: int = 4):
    """Scheme 2: pass p embeds the next bits on lattice p of the running stego (truncating to
    its capacity); returns (stego rows, [per-pass side dicts])."""
    out, sides, pos = [list(r) for r in img], [], 0
    for p in range(passes):
        out, side = embed(out, bits[pos:], T, maxval, truncate=True, lattice=p)
        pos += side["L"]
        sides.append(side)
    return out, sides


def extract_multi(stego, sides):
    """Passes in reverse; the bits in pass order."""
    out, parts = [list(r) for r in stego], []
    for side in reversed(sides):
        b, out = extract(out, side)
        parts.append(b)
    return [b for part in reversed(parts) for b in part], out
