"""Synthetic slice and payload generators.

"ct12": a smooth 12-bit CT-like field plus Gaussian noise, clipped to [0, 4095].
"u16":  uniform uint16 noise (the worst case for the value histogram).
Both are seeded per slice index so that every slice is distinct.
"""
from __future__ import annotations

import random

import numpy as np


def ct12(h: int, w: int, seed: int) -> np.ndarray:
    """(sin(x/97+seed) + cos(y/61) + 2)/4 * 4095 * 0.8 + N(0,16), clip [0,4095], uint16."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = (np.sin(x / 97.0 + seed) + np.cos(y / 61.0) + 2.0) / 4.0 * 4095.0 * 0.8
    img = base + rng.normal(0.0, 16.0, size=(h, w))
    return np.clip(np.rint(img), 0, 4095).astype(np.uint16)


def u16(h: int, w: int, seed: int) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 65536, size=(h, w), dtype=np.uint16)


def u8(h: int, w: int, seed: int) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, size=(h, w), dtype=np.uint8)


GENERATORS = {"ct12": ct12, "u16": u16, "u8": u8}


def payload(nchars: int, seed: int) -> str:
    """Printable-ASCII payload: chr(randrange(32,127)) from random.Random(seed)."""
    r = random.Random(seed)
    return "".join(chr(r.randrange(32, 127)) for _ in range(nchars))


def ct12_torch(b: int, h: int, w: int, device, seed: int = 0):
    """Device-side ct12-like batch for the benchmark (same field, torch RNG noise):
    avoids shipping GBs from the host.  Not bit-identical to `ct12`; parity tests use
    the numpy generator."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    ys = torch.arange(h, device=device, dtype=torch.float32).view(1, h, 1)
    xs = torch.arange(w, device=device, dtype=torch.float32).view(1, 1, w)
    out = torch.empty((b, h, w), dtype=torch.int16, device=device)
    for i in range(b):
        base = (torch.sin(xs / 97.0 + (seed + i)) + torch.cos(ys / 61.0) + 2.0) / 4.0 * 4095.0 * 0.8
        noise = torch.randn((1, h, w), generator=g, device=device) * 16.0
        out[i] = torch.clamp(torch.round(base + noise), 0, 4095).to(torch.int16)[0]
    return out
