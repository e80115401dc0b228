"""CPU oracle: numpy restatement of the reference's stego-quality metrics (src/mse.py).

TEST INFRASTRUCTURE ONLY (same rules as ref_cpu.py): only tests/ may import it, as the
checker for the HIP quality kernel (`codec_quality_moments`) and its host-side math
(`codec_tcc_amd.quality`).

Pinning: checked against golden vectors that tests/golden/make_quality_golden.py made by
importing the reference's `AnalisadorMSE` (mse.py, pydicom stubbed) in the build
container (tests/golden/quality.npz, tests/test_quality.py).

Reference: wesleyfn/codec-tcc @ 2025-10-17, src/mse.py.  Array inputs only (the
reference's file loading, mse.py:13-72, is I/O, not metric arithmetic): for an array,
the reference takes max_val = array.max() (mse.py:85-87, 91-93, 142-143, 148-149).
"""
from __future__ import annotations

from typing import Dict

import numpy as np


def _maxes(a, b, max_value):
    # array branch: each image's own max (mse.py:85-87, 91-93); file branch: the container's
    # full scale for both (DICOM BitsStored, mse.py:31-32; PNG 8/16 bit, :44-55)
    if max_value is None:
        return a.max(), b.max()
    return max_value, max_value


def calcular_mse(img1: np.ndarray, img2: np.ndarray, max_value=None):
    """mse.py:74-117: (mse, max_range)."""
    a = np.array(img1, dtype=np.float64)
    b = np.array(img2, dtype=np.float64)
    m1, m2 = _maxes(a, b, max_value)
    if a.shape != b.shape:                                   # mse.py:98-99
        raise ValueError(f"Dimensões diferentes: {a.shape} vs {b.shape}")
    if m1 != m2:                                             # mse.py:102-107
        r = max(m1, m2)
        an = (a / m1) * r
        bn = (b / m2) * r
    else:
        an, bn, r = a, b, m1
    d = an - bn                                              # mse.py:114-115
    return np.mean(d ** 2), r


def calcular_psnr(mse, max_valor=None):
    """mse.py:119-133."""
    if mse == 0:
        return float("inf")
    if max_valor is None:
        max_valor = 255
    return 10 * np.log10((max_valor ** 2) / mse)


def calcular_ssim_simples(img1: np.ndarray, img2: np.ndarray, max_value=None):
    """mse.py:135-177: one global SSIM window."""
    a = np.array(img1, dtype=np.float64)
    b = np.array(img2, dtype=np.float64)
    m1, m2 = _maxes(a, b, max_value)
    r = max(m1, m2)
    if m1 != m2:
        an = (a / m1) * r
        bn = (b / m2) * r
    else:
        an, bn = a, b
    mu1, mu2 = np.mean(an), np.mean(bn)
    s1, s2 = np.var(an), np.var(bn)
    s12 = np.mean((an - mu1) * (bn - mu2))
    c1 = (0.01 * r) ** 2
    c2 = (0.03 * r) ** 2
    num = (2 * mu1 * mu2 + c1) * (2 * s12 + c2)
    den = (mu1 ** 2 + mu2 ** 2 + c1) * (s1 + s2 + c2)
    return num / den


def difference_stats(img1: np.ndarray, img2: np.ndarray) -> Dict[str, float]:
    """mse.py:201-207: on the raw (unnormalised) float64 arrays."""
    a = np.array(img1, dtype=np.float64)
    b = np.array(img2, dtype=np.float64)
    d = np.abs(a - b)
    nd = int(np.sum(a != b))
    return {"diferenca_media": float(np.mean(d)), "diferenca_max": float(np.max(d)),
            "pixels_diferentes": nd, "percentual_mudanca": nd / a.size * 100}


def analisar_par(img1: np.ndarray, img2: np.ndarray, max_value=None) -> Dict[str, float]:
    """The metric part of analisar_par_imagens (mse.py:179-246) for two arrays."""
    mse, r = calcular_mse(img1, img2, max_value)
    out = {"mse": float(mse), "max_range": float(r), "psnr": float(calcular_psnr(mse, r)),
           "ssim": float(calcular_ssim_simples(img1, img2, max_value))}
    out.update(difference_stats(img1, img2))
    return out


def moments(img1: np.ndarray, img2: np.ndarray) -> Dict[str, int]:
    """The exact integer moments the HIP kernel accumulates (checker for its output)."""
    a = np.asarray(img1).astype(np.int64).ravel()
    b = np.asarray(img2).astype(np.int64).ravel()
    d = np.abs(a - b)
    return {"sum_a": int(a.sum()), "sum_b": int(b.sum()), "sum_aa": int((a * a).sum()),
            "sum_bb": int((b * b).sum()), "sum_ab": int((a * b).sum()), "sum_absdiff": int(d.sum()),
            "max_absdiff": int(d.max()) if d.size else 0, "ndiff": int((a != b).sum()),
            "max_a": int(a.max()) if a.size else 0, "max_b": int(b.max()) if b.size else 0}
