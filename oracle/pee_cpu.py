"""CPU oracle for MED-predictor prediction-error expansion.

TEST INFRASTRUCTURE ONLY (same rules as ref_cpu.py).

PARITY UNPINNED: the reference repository names PEE (README.md:3) but contains no PEE
code, so there is nothing to be bit-exact against.  This module is the
specification of the build's own scheme; the HIP path is checked bit-exact against it,
and the scheme against itself by reversibility (encode -> decode is the identity on the
payload and on the cover).

Scheme (integer only):
  candidates  pixels (y, x) with y = 2i+1, x = 2j+1 (i < H//2, j < W//2), index k = i*(W//2)+j.
              Their MED neighbours a = W(y, x-1), b = N(y-1, x), c = NW(y-1, x-1) all have an
              even coordinate, so they are never modified: prediction at decode time uses
              the same values, and every candidate can be processed independently.
  predictor   MED / LOCO-I: c >= max(a,b) -> min(a,b); c <= min(a,b) -> max(a,b); else a+b-c
  error       e = x - pred
  expansion   -T <= e < T  : x' = pred + 2e + bit         (one payload bit)
  shifting    e >= T       : x' = x + T ;  e < -T : x' = x - T
  overflow    a candidate whose transform could leave [0, maxval] is left unchanged and
              flagged in the location map (LM)
  cursor      payload bit j goes to the j-th expandable, non-overflow candidate in index
              order; processing stops at that candidate for j = L-1 ("end"); candidates
              after `end` are untouched.  Side information: T, L, end, maxval, LM[0..end].
  overflow of the payload (L > capacity): with truncate=True the first `capacity` bits are
              embedded and end = the last candidate (every candidate is processed), status 1;
              the slice stays exactly reversible.  A single streaming pass cannot know
              that no expandable candidate follows, so this -- not "stop at the last
              expandable one" -- is the definition the GPU kernels implement.
  decoding    e' = x' - pred; LM -> unchanged; -2T <= e' < 2T -> bit = e' & 1,
              x = pred + (e' >> 1); e' >= 2T -> x = x' - T; else x = x' + T.

Scheme 2, four sublattice passes (the version-16 container's scheme byte 2):
  lattices    pass 0 (odd, odd) -- scheme 1's candidates; pass 1 (even, even); pass 2 (odd, even);
              pass 3 (even, odd), as (row, column) parities, with y >= 1 and x >= 1 (so every
              candidate has its W / N / NW neighbours).  Each lattice's three MED neighbours lie on
              the other three lattices, so one pass never reads a pixel it writes.
              Lattice (ry, rx): y = 2i + y0, x = 2j + x0, y0 = 1 if ry else 2, x0 = 1 if rx else
              2, i < hc = (H - y0 + 1) // 2, j < wc = (W - x0 + 1) // 2, index k = i * wc + j.
  embed       pass p runs scheme 1 on lattice p of the RUNNING stego (passes 0..p-1 applied),
              truncating to its capacity: it takes the next min(remaining, capacity_p) payload
              bits (all candidates processed when it fills up, as scheme 1's truncation).
              Side information per pass (T, L_p, end_p, LM_p); status 1 when bits remain after
              pass 3.
  decoding    passes 3..0 in reverse, each on the image the later passes' decoding restored:
              pass p's neighbours then hold exactly the values they had when pass p embedded
              (lattices < p still carry their stego values, lattices > p are restored).  The
              payload is the concatenation of the passes' bits in pass order.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np


# (row parity, column parity) of pass p's candidates (scheme 2); lattice 0 is scheme 1's
LATTICES = ((1, 1), (0, 0), (1, 0), (0, 1))


def lattice_origin(lattice: int, H: int, W: int):
    """(y0, x0, hc, wc): lattice candidate (i, j) is pixel (y0 + 2i, x0 + 2j), i < hc, j < wc."""
    ry, rx = LATTICES[lattice]
    y0, x0 = (1 if ry else 2), (1 if rx else 2)
    return y0, x0, max(0, (H - y0 + 1) // 2), max(0, (W - x0 + 1) // 2)


def _grids(img: np.ndarray, lattice: int = 0):
    H, W = img.shape
    y0, x0, hc, wc = lattice_origin(lattice, H, W)
    ys, xs = slice(y0, y0 + 2 * hc, 2), slice(x0, x0 + 2 * wc, 2)
    ys1, xs1 = slice(y0 - 1, y0 - 1 + 2 * hc, 2), slice(x0 - 1, x0 - 1 + 2 * wc, 2)
    x = img[ys, xs].astype(np.int64)
    a = img[ys, xs1].astype(np.int64)
    b = img[ys1, xs].astype(np.int64)
    c = img[ys1, xs1].astype(np.int64)
    return x, a, b, c


def med(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    lo = np.minimum(a, b)
    hi = np.maximum(a, b)
    return np.where(c >= hi, lo, np.where(c <= lo, hi, a + b - c))


def classify(x, p, T: int, maxval: int):
    e = x - p
    expand = (e >= -T) & (e < T)
    right = e >= T
    safe = np.where(expand, (p + 2 * e >= 0) & (p + 2 * e + 1 <= maxval),
                    np.where(right, x + T <= maxval, x - T >= 0))
    return e, expand, right, safe


def pee_embed(cover: np.ndarray, bits: np.ndarray, T: int = 2, maxval: int | None = None,
              truncate: bool = False, lattice: int = 0) -> Tuple[np.ndarray, Dict]:
    if cover.dtype not in (np.uint8, np.uint16) or cover.ndim != 2:
        raise ValueError("cover must be a 2-D uint8/uint16 image")
    if T < 1:
        raise ValueError("T must be >= 1")
    maxval = int(np.iinfo(cover.dtype).max) if maxval is None else int(maxval)
    bits = np.asarray(bits, dtype=np.uint8).ravel()
    L = bits.size
    x, a, b, c = _grids(cover, lattice)
    p = med(a, b, c)
    e, expand, right, safe = classify(x, p, T, maxval)
    es = (expand & safe).ravel()
    capacity = int(es.sum())
    status = 0
    if capacity < L:
        if not truncate:
            raise ValueError(f"payload of {L} bits exceeds the capacity {capacity} at T={T}")
        bits, L, status = bits[:capacity], capacity, 1
        end = es.size - 1
    else:
        end = int(np.flatnonzero(es)[L - 1]) if L else -1
    k = np.arange(es.size)
    proc = (k <= end) & safe.ravel()
    cursor = np.cumsum(es) - 1
    bit = np.zeros(es.size, np.int64)
    bit[es & proc] = bits[cursor[es & proc]]
    xf, pf, ef = x.ravel(), p.ravel(), e.ravel()
    rf = right.ravel()
    new = np.where(es, pf + 2 * ef + bit, np.where(rf, xf + T, xf - T))
    out = np.where(proc, new, xf)
    stego = cover.copy()
    y0, x0, hc, wc = lattice_origin(lattice, *cover.shape)
    stego[y0:y0 + 2 * hc:2, x0:x0 + 2 * wc:2] = out.reshape(hc, wc).astype(cover.dtype)
    lm = ~safe.ravel()[: end + 1]
    return stego, {"T": T, "L": L, "end": end, "maxval": maxval, "lm": lm, "capacity": capacity, "status": status,
                   "lattice": lattice}


def pee_extract(stego: np.ndarray, side: Dict) -> Tuple[np.ndarray, np.ndarray]:
    T, end, L = side["T"], side["end"], side["L"]
    lattice = side.get("lattice", 0)
    x, a, b, c = _grids(stego, lattice)
    p = med(a, b, c).ravel()
    xf = x.ravel()
    e2 = xf - p
    k = np.arange(xf.size)
    lm = np.zeros(xf.size, bool)
    lm[: end + 1] = side["lm"]
    act = (k <= end) & ~lm
    inner = act & (e2 >= -2 * T) & (e2 < 2 * T)
    bits = (e2[inner] & 1).astype(np.uint8)[:L]
    rec = np.where(inner, p + (e2 >> 1), np.where(act & (e2 >= 2 * T), xf - T, np.where(act, xf + T, xf)))
    cover = stego.copy()
    y0, x0, hc, wc = lattice_origin(lattice, *stego.shape)
    cover[y0:y0 + 2 * hc:2, x0:x0 + 2 * wc:2] = rec.reshape(hc, wc).astype(stego.dtype)
    return bits, cover


def pee_embed_multi(cover: np.ndarray, bits: np.ndarray, T: int = 2, maxval: int | None = None,
                    passes: int = 4) -> Tuple[np.ndarray, Dict]:
    """Scheme 2: passes 0..passes-1 on lattices 0..passes-1 of the running stego, each taking
    the next min(remaining, capacity) bits.  Side: T, L (bits embedded), status (1: bits left
    over), and the per-pass side dicts."""
    if not 1 <= passes <= 4:
        raise ValueError("passes must be in 1..4")
    bits = np.asarray(bits, dtype=np.uint8).ravel()
    stego, sides, pos = cover.copy(), [], 0
    for p in range(passes):
        stego, side = pee_embed(stego, bits[pos:], T, maxval, truncate=True, lattice=p)
        pos += side["L"]
        sides.append(side)
    return stego, {"T": T, "L": pos, "status": 1 if pos < bits.size else 0, "passes": sides,
                   "maxval": sides[0]["maxval"]}


def pee_extract_multi(stego: np.ndarray, side: Dict) -> Tuple[np.ndarray, np.ndarray]:
    """Inverse of pee_embed_multi: passes in reverse, bits concatenated in pass order."""
    img, got = stego, []
    for ps in reversed(side["passes"]):
        b, img = pee_extract(img, ps)
        got.append(b)
    return (np.concatenate(got[::-1]) if got else np.zeros(0, np.uint8)), img


def capacity_curve(cover: np.ndarray, tmax: int, maxval: int | None = None) -> np.ndarray:
    """Capacities at T = 1..tmax.  The expansion safety test does not depend on T, so the
    curve is a cumulative count of prediction errors e in [-T, T) over the candidates whose
    expansion stays in [0, maxval] (this is what codec_pee_capacity computes)."""
    maxval = int(np.iinfo(cover.dtype).max) if maxval is None else int(maxval)
    x, a, b, c = _grids(cover)
    p = med(a, b, c)
    e = (x - p).ravel()
    p = p.ravel()
    ok = (p + 2 * e >= 0) & (p + 2 * e + 1 <= maxval)
    return np.array([int((ok & (e >= -T) & (e < T)).sum()) for T in range(1, tmax + 1)], dtype=np.int64)


def select_T(cover: np.ndarray, L: int, tmax: int = 16, maxval: int | None = None) -> int:
    """The smallest T <= tmax whose capacity holds L bits (tmax if none does)."""
    curve = capacity_curve(cover, tmax, maxval)
    hit = np.flatnonzero(curve >= L)
    return int(hit[0]) + 1 if hit.size else tmax


def capacity(cover: np.ndarray, T: int = 2, maxval: int | None = None, lattice: int = 0) -> int:
    maxval = int(np.iinfo(cover.dtype).max) if maxval is None else int(maxval)
    x, a, b, c = _grids(cover, lattice)
    _e, expand, _r, safe = classify(x, med(a, b, c), T, maxval)
    return int((expand & safe).sum())
