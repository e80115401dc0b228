#!/usr/bin/env python3
"""Golden vectors for the stego-quality metrics (reference src/mse.py, class AnalisadorMSE).

Run in the BUILD container only (reads /root/reference):

    python tests/golden/make_quality_golden.py

The reference module imports pydicom at top (mse.py:7); a stub module is registered so it
loads (the metric methods never touch it).  Two reference entry modes are recorded:
  * array mode: calcular_mse / calcular_psnr / calcular_ssim_simples called with numpy
    arrays (max_val = array max, mse.py:85-93);
  * file mode: analisar_par_imagens on PNG files written here (8-bit 'L' and 16-bit
    'I;16'; max_val = the format's full scale, mse.py:42-55), which also yields the
    difference statistics (mse.py:201-207).
Only data (inputs and the reference's outputs) is written: tests/golden/quality.npz.
"""
from __future__ import annotations

import contextlib
import importlib.util
import io
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from codec_tcc_amd import synth  # noqa: E402


def load_reference():
    sys.modules.setdefault("pydicom", types.ModuleType("pydicom"))
    spec = importlib.util.spec_from_file_location("ref_mse", "/root/reference/src/mse.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pairs():
    sys.path.insert(0, os.path.dirname(HERE))
    import golden_io
    out = []
    # real images from the LSB golden cases: cover vs the reference's stego
    for case in golden_io.cases():
        if case["name"] in ("pe_b0.4_1k", "torax_b0.4_1k"):
            out.append((case["name"], case["cover"], golden_io.stego(case)))
    rng = np.random.default_rng(11)
    c = synth.ct12(192, 160, 3)
    s = c.copy()
    idx = rng.choice(c.size, 700, replace=False)
    s.flat[idx] ^= 1
    out.append(("ct12_lsb700", c, s))
    # the maximum pixel loses 1: maxima differ -> the normalisation branch (mse.py:102-107)
    c2 = c.copy()
    s2 = c2.copy()
    s2.flat[int(np.argmax(c2))] -= 1
    s2.flat[idx[:50]] ^= 1
    out.append(("ct12_maxdrop", c2, s2))
    u = synth.u16(96, 128, 5)
    out.append(("u16_noise", u, (u.astype(np.int64) + rng.integers(-3, 4, u.shape)).clip(0, 65535).astype(np.uint16)))
    g = (rng.integers(0, 256, (80, 72))).astype(np.uint8)
    out.append(("u8_identical", g, g.copy()))
    g2 = g.copy()
    g2[::7, ::5] ^= 3
    out.append(("u8_sparse", g, g2))
    return out


def main():
    ref = load_reference()
    an = ref.AnalisadorMSE()
    data = {}
    names = []
    quiet = contextlib.redirect_stdout(io.StringIO())
    with tempfile.TemporaryDirectory() as td, quiet:
        from PIL import Image
        for name, a, b in pairs():
            names.append(name)
            if name not in ("pe_b0.4_1k", "torax_b0.4_1k"):   # those two come from cases.npz
                data[f"{name}__a"] = a
                data[f"{name}__b"] = b
            mse, r = an.calcular_mse(a, b)
            data[f"{name}__arr"] = np.array([mse, r, an.calcular_psnr(mse, r), an.calcular_ssim_simples(a, b)],
                                            np.float64)
            pa, pb = os.path.join(td, f"{name}_a.png"), os.path.join(td, f"{name}_b.png")
            Image.fromarray(a).save(pa)
            Image.fromarray(b).save(pb)
            res = an.analisar_par_imagens(pa, pb, name)
            data[f"{name}__file"] = np.array([res["mse"], res["psnr"], res["ssim"], res["diferenca_media"],
                                              res["diferenca_max"], res["percentual_mudanca"]], np.float64)
    data["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "quality.npz"), **data)
    print(f"wrote {len(names)} quality cases")


if __name__ == "__main__":
    main()
