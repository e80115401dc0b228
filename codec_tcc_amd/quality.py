"""Stego-quality metrics of the reference's src/mse.py on the MI355X.

The reference (class AnalisadorMSE) computes MSE, PSNR, a single-window SSIM and
difference statistics with float64 numpy over whole images.  Here one read-only HIP pass
(`codec_quality_moments`, csrc/codec_quality.hip) produces exact integer moments per
slice, and every metric is evaluated from them in exact rational arithmetic
(`fractions.Fraction`) with one final rounding.  The values agree with the reference's to
float64 rounding noise (tests/test_quality.py pins them against golden outputs of the
reference itself), and are the correctly rounded exact values.

    q = quality(covers, stegos)                 # torch [B,H,W] on the GPU -> list of dicts
    q = quality(covers, stegos, max_value=4095) # "file mode": declared full scale (BitsStored)
    AnalisadorMSE().calcular_mse(img1, img2)     # drop-in for mse.py:74 (arrays / tensors)
"""
from __future__ import annotations

import math
from fractions import Fraction
from typing import Dict, List, Optional

import numpy as np

from . import _lib
from .codec import _elem_bytes, _require_gpu, _stream, _torch

WORDS = 10
KEYS = ("sum_a", "sum_b", "sum_aa", "sum_bb", "sum_ab", "sum_absdiff", "max_absdiff", "ndiff", "max_a", "max_b")


def moments(a, b) -> np.ndarray:
    """Exact per-slice moments of two [B,H,W] (or [H,W]) uint8/uint16 GPU tensors:
    uint64 [B, 10] in the order of KEYS (include/codec_tcc.h, codec_quality_moments)."""
    _require_gpu()
    torch = _torch()
    if tuple(a.shape) != tuple(b.shape):
        raise ValueError(f"Dimensões diferentes: {tuple(a.shape)} vs {tuple(b.shape)}")   # mse.py:98-99
    if a.dtype != b.dtype:
        raise TypeError("both images must have the same dtype")
    if a.dim() == 2:
        a, b = a.unsqueeze(0), b.unsqueeze(0)
    if a.dim() != 3:
        raise ValueError("expected [B,H,W] or [H,W]")
    nb = _elem_bytes(a)
    a, b = a.contiguous(), b.contiguous()
    B, H, W = (int(x) for x in a.shape)
    out = torch.empty((B, WORDS), dtype=torch.int64, device=a.device)
    _lib.check(_lib.load().codec_quality_moments(B, H, W, nb, a.data_ptr(), b.data_ptr(), out.data_ptr(), _stream()),
               "codec_quality_moments")
    return out.cpu().numpy().view(np.uint64)


def _f(x: Fraction) -> float:
    return x.numerator / x.denominator   # correctly rounded (Python int true division)


def metrics_from_moments(m, npx: int, max_value: Optional[float] = None) -> Dict[str, float]:
    """mse.py metrics from one slice's exact moments.

    max_value None -> array mode (mse.py:85-93: each image's max is its own max_val, and
    the two are rescaled to the larger when they differ, :102-107); a number -> file
    mode (both images carry the container's full scale, :31-32 / :44-55)."""
    d = {k: int(v) for k, v in zip(KEYS, m)}
    N = Fraction(npx)
    if max_value is None:
        m1, m2 = d["max_a"], d["max_b"]
    else:
        m1 = m2 = max_value
    r = max(m1, m2)
    if m1 != m2:
        if m1 == 0 or m2 == 0:
            nan = float("nan")
            return {"mse": nan, "max_range": float(r), "psnr": nan, "ssim": nan, **_diffs(d, npx)}
        k1, k2 = Fraction(r) / Fraction(m1), Fraction(r) / Fraction(m2)
    else:
        k1 = k2 = Fraction(1)
    saa, sbb, sab = Fraction(d["sum_aa"]), Fraction(d["sum_bb"]), Fraction(d["sum_ab"])
    sa, sb = Fraction(d["sum_a"]), Fraction(d["sum_b"])
    # calcular_mse (mse.py:114-115): mean((k1 a - k2 b)^2)
    mse = (k1 * k1 * saa - 2 * k1 * k2 * sab + k2 * k2 * sbb) / N
    mse_f = _f(mse)
    # calcular_psnr (mse.py:127-133)
    rf = float(r)
    psnr = float("inf") if mse == 0 else 10 * math.log10((rf ** 2) / mse_f)
    # calcular_ssim_simples (mse.py:160-175): one global window
    mu1, mu2 = k1 * sa / N, k2 * sb / N
    v1 = k1 * k1 * (saa / N - (sa / N) ** 2)
    v2 = k2 * k2 * (sbb / N - (sb / N) ** 2)
    c12 = k1 * k2 * (sab / N - (sa / N) * (sb / N))
    c1 = Fraction((0.01 * rf) ** 2)       # the reference's float constants, taken exactly
    c2 = Fraction((0.03 * rf) ** 2)
    num = (2 * mu1 * mu2 + c1) * (2 * c12 + c2)
    den = (mu1 ** 2 + mu2 ** 2 + c1) * (v1 + v2 + c2)
    ssim = _f(num / den) if den != 0 else float("nan")
    return {"mse": mse_f, "max_range": rf, "psnr": psnr, "ssim": ssim, **_diffs(d, npx)}


def _diffs(d, npx: int) -> Dict[str, float]:
    """mse.py:201-207 on the raw arrays."""
    return {"diferenca_media": _f(Fraction(d["sum_absdiff"], npx)), "diferenca_max": float(d["max_absdiff"]),
            "pixels_diferentes": d["ndiff"], "percentual_mudanca": _f(Fraction(d["ndiff"] * 100, npx))}


def quality(covers, stegos, max_value: Optional[float] = None) -> List[Dict[str, float]]:
    """Per-slice mse / max_range / psnr / ssim / difference statistics of a batch."""
    mom = moments(covers, stegos)
    npx = int(covers.shape[-1]) * int(covers.shape[-2])
    return [metrics_from_moments(mom[i], npx, max_value) for i in range(mom.shape[0])]


class AnalisadorMSE:
    """Drop-in for the metric methods of the reference's AnalisadorMSE (mse.py:9),
    taking arrays or GPU tensors (file loading is codec_tcc_amd.dicom's business)."""

    def __init__(self):
        self.resultados = []

    @staticmethod
    def _pair(img1, img2):
        torch = _torch()
        a = img1 if isinstance(img1, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(img1))
        b = img2 if isinstance(img2, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(img2))
        dev = torch.device("cuda", torch.cuda.current_device())
        return a.to(dev), b.to(dev)

    def calcular_mse(self, imagem1, imagem2):
        """mse.py:74-117 -> (mse, max_range)."""
        a, b = self._pair(imagem1, imagem2)
        q = quality(a, b)[0]
        return q["mse"], q["max_range"]

    @staticmethod
    def calcular_psnr(mse, max_valor=None):
        """mse.py:119-133."""
        if mse == 0:
            return float("inf")
        if max_valor is None:
            max_valor = 255
        return 10 * math.log10((max_valor ** 2) / mse)

    def calcular_ssim_simples(self, imagem1, imagem2):
        """mse.py:135-177."""
        a, b = self._pair(imagem1, imagem2)
        return quality(a, b)[0]["ssim"]

    def analisar_par(self, imagem1, imagem2, nome_par: str = "", max_value: Optional[float] = None):
        """The metric dict of analisar_par_imagens (mse.py:179-246) for two images."""
        a, b = self._pair(imagem1, imagem2)
        r = dict(quality(a, b, max_value)[0])
        r["nome"] = nome_par
        self.resultados.append(r)
        return r

