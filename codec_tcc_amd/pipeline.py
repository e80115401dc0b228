"""File-level pipeline around the GPU path: the reference's main() encode (codec.py:847-913)
and decode_bin() (codec.py:795-842), with the STGC container and the DICOM reader/writer.

The pixel work (decomposition, block search, embedding, bitmaps, extraction) runs on the
MI355X through the C ABI; this module only moves bytes (zlib, struct, files).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
from typing import Dict, Optional, Tuple

import numpy as np

from . import api, container, dicom
from .codec import Codec, _require_gpu, _torch, meta_records


def _compress(stego: np.ndarray, codec: str) -> bytes:
    if codec == "raw":
        return container.encode_stego_raw(stego)
    if codec == "jxl":   # codec.py:111-129 (cjxl -d 0 -e 3: lossless), only where the binary exists
        exe = shutil.which("cjxl") or shutil.which("cjxl.exe")
        if not exe:
            raise RuntimeError("codec 'jxl' needs the cjxl binary on PATH (absent on this image)")
        from PIL import Image
        with tempfile.TemporaryDirectory() as d:
            png, jxl = os.path.join(d, "in.png"), os.path.join(d, "out.jxl")
            Image.fromarray(stego.astype(np.uint16)).save(png)
            subprocess.run([exe, png, jxl, "-d", "0", "-e", "3"], check=True, capture_output=True)
            return open(jxl, "rb").read()
    raise ValueError(f"Codec '{codec}' não suportado.")   # codec.py:165


def _decompress(data: bytes, codec: str, height: int, width: int) -> np.ndarray:
    if codec in ("raw", "unknown"):
        return container.decode_stego_raw(data, height, width)
    if codec == "jxl":   # codec.py:169-182
        exe = shutil.which("djxl") or shutil.which("djxl.exe")
        if not exe:
            raise RuntimeError("codec 'jxl' needs the djxl binary on PATH (absent on this image)")
        from PIL import Image
        with tempfile.TemporaryDirectory() as d:
            jxl, png = os.path.join(d, "in.jxl"), os.path.join(d, "out.png")
            open(jxl, "wb").write(data)
            subprocess.run([exe, jxl, png], check=True, capture_output=True)
            with Image.open(png) as im:
                return np.array(im)
    raise ValueError(f"Codec '{codec}' não suportado.")   # codec.py:209


def encode_file(image, message: str, out_path: str, *, beta: float = 0.4, block: int = 16,
                codec: str = "raw", version: Optional[int] = None) -> Dict:
    """main() (codec.py:856-909): load -> decompose (beta) -> hybrid embed (block) -> merge
    -> stego codec -> zlib(bitmaps) -> header -> .bin.  `image` is an array or a DICOM path.
    version None: 1 (reference layout, start_offset written as 0 like codec.py:903) when the
    fields fit 16 bits, else 2 (32-bit fields, real offset)."""
    _require_gpu()
    torch = _torch()
    img = image if isinstance(image, np.ndarray) else dicom.read_dicom(image)[0]
    if img.ndim != 2 or img.dtype not in (np.uint8, np.uint16):
        raise ValueError("A imagem deve ser 2D uint8 ou uint16.")
    h, w = img.shape
    c = Codec(1, h, w, dtype=str(img.dtype), beta=beta, block=block)
    enc = c.encode(torch.from_numpy(np.ascontiguousarray(img)[None]).cuda(), [message])
    m = meta_records(enc.meta)[0]
    s = m.s
    dense = c.expand_maps(enc.maps, enc.meta, map_words=enc.payloads.map_words, smax=s).cpu().numpy()[0]
    stego = enc.stego.cpu().numpy()[0]
    blob = container.bitmaps_blob(dense)
    sizes = [m.sizes[p] for p in range(s)]
    perm = [m.perm[j] for j in range(s)]
    fits16 = w <= 0xFFFF and h <= 0xFFFF and all(0 <= x <= 0xFFFF for x in sizes)
    ver = version if version is not None else (1 if fits16 else 2)
    hdr = container.create_header(codec, s, sizes, perm, len(blob), w, h, 0 if ver == 1 else m.start_offset,
                                  False, version=ver)
    size = container.create_binary_file(out_path, hdr, _compress(stego, codec), blob)
    return {"path": out_path, "bytes": size, "version": ver, "s": s, "segments_lengths": sizes,
            "segment_indices": perm, "start_offset": m.start_offset, "stego": stego}


def decode_bin(filepath: str, output_prefix: Optional[str] = None) -> Tuple[str, np.ndarray]:
    """decode_bin (codec.py:795-842): the reference's message (its lossy decode_message,
    bit-exact) and the stego image.  Files are written only when output_prefix is given."""
    md, blob, payload = container.parse_bin_file(filepath)
    s = md["s"]
    stego = _decompress(payload, md["codec"], md["height"], md["width"])
    bitmaps = container.split_bitmaps(blob, s)
    message = api.decode_message(api.extract_local_planes(stego, s), bitmaps, md)
    if output_prefix is not None:
        with open(f"{output_prefix}_mensagem.txt", "w", encoding="utf-8") as f:
            f.write(message)
        dicom.save_dicom(stego, f"{output_prefix}_imagem.dcm")
    return message, stego


def decode_bin_exact(filepath: str, search_block_size: int = 16) -> Tuple[str, np.ndarray]:
    """Exact payload bits and the restored cover from a .bin."""
    md, blob, payload = container.parse_bin_file(filepath)
    s = md["s"]
    stego = _decompress(payload, md["codec"], md["height"], md["width"])
    bitmaps = container.split_bitmaps(blob, s)
    return api.decode_positional(stego, bitmaps, md, search_block_size=search_block_size,
                                 align_across_planes=bool(md["align_flag"]))
