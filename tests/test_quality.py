"""Stego-quality metrics (reference src/mse.py): oracle vs the reference's own outputs,
the exact-moment host math vs the same, and (GPU) the HIP moments kernel vs the oracle."""
import math

import numpy as np
import pytest

import golden_io
from codec_tcc_amd import quality as Q
from codec_tcc_amd import synth
from oracle import quality_cpu as O

QC = golden_io.quality_cases()
IDS = [c["name"] for c in QC]


def _full_scale(a):
    return 65535.0 if a.dtype == np.uint16 else 255.0     # PNG 'I;16' / 'L' (mse.py:44-55)


def _close(x, y, rtol=1e-12):
    if math.isinf(y) or math.isnan(y):
        return (math.isinf(x) and x == y) or (math.isnan(x) and math.isnan(y))
    return abs(x - y) <= rtol * max(abs(y), 1e-300) + 1e-300


@pytest.mark.parametrize("c", QC, ids=IDS)
def test_oracle_matches_reference(c):
    mse, r = O.calcular_mse(c["a"], c["b"])
    assert [mse, r, O.calcular_psnr(mse, r), O.calcular_ssim_simples(c["a"], c["b"])] == list(c["arr"])
    fs = _full_scale(c["a"])
    got = O.analisar_par(c["a"], c["b"], max_value=fs)
    exp = c["file"]
    assert got["mse"] == exp[0] and got["ssim"] == exp[2]
    assert got["psnr"] == exp[1] or (math.isinf(got["psnr"]) and math.isinf(exp[1]))
    assert [got["diferenca_media"], got["diferenca_max"], got["percentual_mudanca"]] == list(exp[3:])


@pytest.mark.parametrize("c", QC, ids=IDS)
def test_moment_math_matches_reference(c):
    """Host side of the GPU path, fed with exact moments computed on the CPU: the closed
    forms reproduce the reference to float64 rounding (rtol 1e-12; psnr/ssim 1e-12)."""
    m = O.moments(c["a"], c["b"])
    mv = [m[k] for k in Q.KEYS]
    npx = c["a"].size
    got = Q.metrics_from_moments(mv, npx)
    mse, r, psnr, ssim = c["arr"]
    assert _close(got["mse"], mse) and got["max_range"] == r
    assert _close(got["psnr"], psnr) and _close(got["ssim"], ssim)
    got = Q.metrics_from_moments(mv, npx, max_value=_full_scale(c["a"]))
    exp = c["file"]
    assert _close(got["mse"], exp[0]) and _close(got["psnr"], exp[1]) and _close(got["ssim"], exp[2])
    assert _close(got["diferenca_media"], exp[3]) and got["diferenca_max"] == exp[4]
    assert _close(got["percentual_mudanca"], exp[5])


def test_moment_math_random_pairs():
    """More shapes/dtypes than the fixtures: host math vs the oracle (itself pinned above)."""
    rng = np.random.default_rng(3)
    for trial in range(12):
        dt = np.uint16 if trial % 2 else np.uint8
        hi = 4096 if dt == np.uint16 else 256
        a = rng.integers(0, hi, (rng.integers(1, 40), rng.integers(1, 40))).astype(dt)
        b = a.copy()
        k = rng.integers(0, a.size + 1)
        b.flat[:k] = rng.integers(0, hi, k).astype(dt)
        if trial % 3 == 0 and a.max() > 0:                 # different maxima: normalisation branch
            b.flat[int(np.argmax(b))] = max(0, int(b.max()) - 1)
        m = O.moments(a, b)
        got = Q.metrics_from_moments([m[k] for k in Q.KEYS], a.size)
        exp = O.analisar_par(a, b)
        for key in ("mse", "psnr", "ssim", "diferenca_media", "percentual_mudanca"):
            with np.errstate(all="ignore"):
                assert _close(got[key], exp[key], 1e-9), (trial, key, got[key], exp[key])
        assert got["diferenca_max"] == exp["diferenca_max"] and got["pixels_diferentes"] == exp["pixels_diferentes"]


@pytest.mark.gpu
@pytest.mark.parametrize("dt,h,w,bsz", [("uint16", 512, 512, 3), ("uint16", 37, 53, 2), ("uint8", 64, 96, 4),
                                        ("uint8", 33, 31, 1), ("uint16", 2048, 2048, 2),
                                        ("u16full", 512, 512, 2), ("u16full", 2048, 2048, 1)])
def test_gpu_moments_exact(dt, h, w, bsz):
    """Exact integer moments; "u16full" = uniform 16-bit noise (products up to 65535^2, the
    kernel's per-thread float64 sums at their largest)."""
    torch = pytest.importorskip("torch")
    gen = {"uint16": synth.ct12, "u16full": synth.GENERATORS["u16"]}.get(dt, synth.GENERATORS["u8"])
    rng = np.random.default_rng(h * w)
    a = np.stack([gen(h, w, 10 + i) for i in range(bsz)])
    b = a.copy()
    for i in range(bsz):
        idx = rng.choice(h * w, min(h * w, 5000), replace=False)
        b[i].flat[idx] ^= np.asarray(rng.integers(0, 4, idx.size), dtype=a.dtype)
    got = Q.moments(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda())
    for i in range(bsz):
        m = O.moments(a[i], b[i])
        assert [int(x) for x in got[i]] == [m[k] for k in Q.KEYS]


@pytest.mark.gpu
@pytest.mark.parametrize("c", QC, ids=IDS)
def test_gpu_quality_matches_reference(c):
    torch = pytest.importorskip("torch")
    ta, tb = torch.from_numpy(c["a"]).cuda(), torch.from_numpy(c["b"]).cuda()
    an = Q.AnalisadorMSE()
    mse, r = an.calcular_mse(ta, tb)
    assert _close(mse, c["arr"][0]) and r == c["arr"][1]
    assert _close(an.calcular_psnr(mse, r), c["arr"][2])
    assert _close(an.calcular_ssim_simples(c["a"], c["b"]), c["arr"][3])
    q = Q.quality(ta, tb, max_value=_full_scale(c["a"]))[0]
    exp = c["file"]
    assert _close(q["mse"], exp[0]) and _close(q["psnr"], exp[1]) and _close(q["ssim"], exp[2])
    assert _close(q["diferenca_media"], exp[3]) and q["diferenca_max"] == exp[4]
