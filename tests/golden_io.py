"""Loaders for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def images():
    z = _load("images.npz")
    return {"pe": z["pe"], "torax": z["torax"]}


def cases():
    """Yield dict per embed case with the image resolved."""
    z = _load("cases.npz")
    imgs = images()
    out = []
    for name in z["__names__"]:
        name = str(name)
        pre = name + "/"
        d = {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}
        d["name"] = name
        key = str(d["image_key"])
        d["cover"] = imgs[key] if key in imgs else d["image"]
        out.append(d)
    return out


def tables():
    return _load("tables.npz")


def kat2048():
    with open(os.path.join(GOLDEN, "kat2048.json")) as f:
        return json.load(f)


def dense_bitmaps(case):
    s = int(case["s"])
    h, w = case["cover"].shape
    bits = np.unpackbits(case["bitmaps_packed"])[: s * h * w]
    return bits.reshape(s, h, w)


def stego(case):
    if "stego_xor" in case:
        return case["cover"] ^ case["stego_xor"]
    return case["stego"]


def decoded(case):
    """decode_message() output (stored as UTF-8 bytes: numpy strings drop trailing NULs)."""
    return case["decoded_utf8"].tobytes().decode("utf-8")


def message(case):
    return case["msg_utf8"].tobytes().decode("utf-8") if "msg_utf8" in case else None


def quality_cases():
    """Stego-quality golden cases (make_quality_golden.py): dicts with a, b and the
    reference's array-mode [mse, max_range, psnr, ssim] and file-mode
    [mse, psnr, ssim, diferenca_media, diferenca_max, percentual_mudanca]."""
    d = _load("quality.npz")
    lsb = {c["name"]: c for c in cases() if c["name"] in ("pe_b0.4_1k", "torax_b0.4_1k")}
    out = []
    for n in d["names"]:
        n = str(n)
        if n in lsb:
            a, b = lsb[n]["cover"], stego(lsb[n])
        else:
            a, b = d[f"{n}__a"], d[f"{n}__b"]
        out.append({"name": n, "a": a, "b": b, "arr": d[f"{n}__arr"], "file": d[f"{n}__file"]})
    return out
