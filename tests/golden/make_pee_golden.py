#!/usr/bin/env python3
"""Known-answer vectors of the MED-PEE scheme -> tests/golden/pee_kat.json (scheme 1, one
pass) and tests/golden/pee_multi_kat.json (scheme 2, four sublattice passes).

Computed by the scalar restatement tests/pee_scalar.py (not by the vectorised oracle they
then check).  Covers: seeded ct12 / u8 / u16 images (and ct12 x 16 as smooth 16-bit data), even and odd sizes, T = 1..5, a
non-default maxval, images pushed to 0 / maxval (overflow location map), payloads of 0 bits,
exactly the capacity, and beyond it (truncated, status 1).  Inputs are regenerated from
their seeds (codec_tcc_amd.synth + numpy default_rng), so the file holds only digests.

    python tests/golden/make_pee_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from codec_tcc_amd import synth  # noqa: E402
import pee_scalar as S  # noqa: E402

# (kind, h, w, seed, T, maxval or None, clip: push pixels to the range ends, payload rule)
CASES = [
    ("ct12", 32, 48, 1, 2, None, False, "half"),
    ("ct12", 33, 41, 2, 1, 4095, False, "half"),
    ("ct12", 40, 40, 3, 3, 4095, True, "cap"),
    ("ct12", 24, 64, 4, 5, 4095, True, "over"),
    ("u8", 30, 32, 5, 2, None, True, "half"),
    ("u8", 31, 33, 6, 1, None, True, "over"),
    ("ct16", 16, 32, 7, 4, None, False, "cap"),
    ("ct12", 20, 24, 8, 2, 4095, False, "zero"),
    ("ct16", 18, 40, 9, 2, 65535, True, "half"),
    ("u16", 16, 24, 10, 3, None, False, "over"),
]


def make_image(kind, h, w, seed, maxval, clip):
    if kind == "ct16":   # 16-bit data that still has small prediction errors
        img = (synth.ct12(h, w, seed).astype(np.uint32) * 16).astype(np.uint16)
    else:
        img = synth.GENERATORS[kind](h, w, seed)
    if clip:   # bands of pixels at the range ends: expansions and shifts that would overflow
        top = int(np.iinfo(img.dtype).max) if maxval is None else int(maxval)
        rng = np.random.default_rng(50 + seed)
        img = img.copy()
        img[: h // 4] = rng.integers(0, 3, (h // 4, w))
        img[h // 4: h // 2] = top - rng.integers(0, 3, (h // 2 - h // 4, w))
    return img


def payload_bits(n, seed):
    return np.random.default_rng(1000 + seed).integers(0, 2, n).astype(np.uint8)


def case_inputs(c):
    kind, h, w, seed, T, maxval, clip, rule = c
    img = make_image(kind, h, w, seed, maxval, clip)
    mv = int(np.iinfo(img.dtype).max) if maxval is None else int(maxval)
    _st, side = S.embed(img.tolist(), [], T, mv)          # capacity at T
    cap = side["capacity"]
    n = {"half": cap // 2, "cap": cap, "over": cap + 25, "zero": 0}[rule]
    return img, payload_bits(n, seed), T, mv


# scheme 2 (four sublattice passes): (kind, h, w, seed, T, maxval, clip, payload rule); rules
# against the scheme's total capacity C (bits a payload longer than every pass can take
# embeds): "pass0" = lattice 0's capacity on the cover (one pass), "two" = that + 3 (spills
# into pass 1), "all" = C (every pass filled), "over" = C + 40 (status 1), "zero"
MULTI_CASES = [
    ("ct12", 32, 48, 11, 2, 4095, False, "two"),
    ("ct12", 33, 41, 12, 1, 4095, False, "all"),
    ("ct12", 24, 31, 13, 3, 4095, True, "over"),
    ("u8", 30, 32, 14, 2, None, True, "two"),
    ("u8", 27, 20, 15, 1, None, False, "pass0"),
    ("ct16", 16, 34, 16, 4, None, False, "all"),
    ("u16", 17, 24, 17, 2, None, True, "over"),
    ("ct12", 20, 24, 18, 2, 4095, False, "zero"),
]


def multi_case_inputs(c):
    kind, h, w, seed, T, maxval, clip, rule = c
    img = make_image(kind, h, w, seed, maxval, clip)
    mv = int(np.iinfo(img.dtype).max) if maxval is None else int(maxval)
    _st, side0 = S.embed(img.tolist(), [], T, mv)
    _st, sides = S.embed_multi(img.tolist(), [1] * (4 * h * w), T, mv)   # every pass filled
    total = sum(sd["L"] for sd in sides)
    n = {"pass0": side0["capacity"], "two": side0["capacity"] + 3, "all": total, "over": total + 40,
         "zero": 0}[rule]
    return img, payload_bits(n, 500 + seed), T, mv


def multi_main():
    out = []
    for c in MULTI_CASES:
        img, bits, T, mv = multi_case_inputs(c)
        st, sides = S.embed_multi(img.tolist(), [int(b) for b in bits], T, mv)
        stego = np.array(st, dtype=img.dtype)
        got, back = S.extract_multi(st, sides)
        L = sum(sd["L"] for sd in sides)
        assert got == [int(b) for b in bits[:L]] and back == img.tolist()
        out.append({"kind": c[0], "h": c[1], "w": c[2], "seed": c[3], "T": T, "maxval": c[5], "clip": c[6],
                    "rule": c[7], "L_in": int(bits.size), "L": L, "status": 1 if L < bits.size else 0,
                    "passes": [{"L": sd["L"], "end": sd["end"], "capacity": sd["capacity"], "status": sd["status"],
                                "lm_hex": np.packbits(np.array(sd["lm"], bool), bitorder="little").tobytes().hex()}
                               for sd in sides],
                    "stego_sha256": hashlib.sha256(stego.tobytes()).hexdigest()})
    with open(os.path.join(HERE, "pee_multi_kat.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out)} cases -> pee_multi_kat.json")


def main():
    out = []
    for c in CASES:
        img, bits, T, mv = case_inputs(c)
        st, side = S.embed(img.tolist(), [int(b) for b in bits], T, mv)
        stego = np.array(st, dtype=img.dtype)
        got, back = S.extract(st, side)
        assert got == [int(b) for b in bits[: side["L"]]] and back == img.tolist()
        out.append({"kind": c[0], "h": c[1], "w": c[2], "seed": c[3], "T": T, "maxval": c[5], "clip": c[6],
                    "rule": c[7], "L_in": int(bits.size), "L": side["L"], "end": side["end"],
                    "capacity": side["capacity"], "status": side["status"],
                    "lm_hex": np.packbits(np.array(side["lm"], bool), bitorder="little").tobytes().hex(),
                    "lm_ones": int(sum(side["lm"])),
                    "stego_sha256": hashlib.sha256(stego.tobytes()).hexdigest()})
    with open(os.path.join(HERE, "pee_kat.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out)} cases -> pee_kat.json")


if __name__ == "__main__":
    main()
    multi_main()
