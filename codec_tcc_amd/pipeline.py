"""File-level pipeline around the GPU path: the reference's main() encode (codec.py:847-913)
and decode_bin() (codec.py:795-842), with the STGC container and the DICOM reader/writer;
plus the same file round trip for the MED-PEE scheme (encode_file_pee / decode_bin_pee).

The pixel work (decomposition, block search, embedding, bitmaps, extraction, MED-PEE) runs
on the MI355X through the C ABI; this module only moves bytes (zlib, struct, files).

Stego codecs (compress_image / decompress_image, codec.py:108-209):
  raw  this build's uncompressed little-endian pixels (container id 0)
  png  the reference's Deflated Explicit VR Little Endian DICOM (codec.py:151-162, 203-206),
       written and read by dicom.py (zlib raw deflate)
  jxl  cjxl -d 0 -e 3 / djxl (codec.py:111-129, 169-182): runs where the binaries exist
  j2k, jls  gdcmconv (codec.py:132-149, 184-201): the binary and a JPEG 2000 / JPEG-LS
       pixel decoder are absent from this image; both raise RuntimeError naming what is missing
"""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
from typing import Dict, Optional, Tuple

import numpy as np

from . import _lib, api, container, dicom, framing
from .codec import Codec, _require_gpu, _torch, meta_records


def _compress(stego: np.ndarray, codec: str) -> bytes:
    if codec == "raw":
        return container.encode_stego_raw(stego)
    if codec == "png":   # codec.py:151-162: create_dicom + DeflatedExplicitVRLittleEndian
        return dicom.create_dicom_bytes(stego, transfer_syntax=dicom.DEFLATED_LE)
    if codec in ("j2k", "jls"):   # codec.py:132-149
        raise RuntimeError(f"codec '{codec}' needs the gdcmconv binary and a JPEG 2000 / JPEG-LS decoder "
                           "(both absent on this image)")
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
    if codec == "png":   # codec.py:203-206: dcmread(force=True).pixel_array
        img = dicom.read_dicom(data)[0]
        if img.shape != (height, width):
            raise ValueError("png (deflated DICOM) stego does not match the header's width x height")
        return img
    if codec in ("j2k", "jls"):   # codec.py:184-201
        raise RuntimeError(f"codec '{codec}' needs the gdcmconv binary and a JPEG 2000 / JPEG-LS decoder "
                           "(both absent on this image)")
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
                                  False, version=ver, search_block_size=block if ver == 2 else None)
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


def decode_bin_exact(filepath: str, search_block_size: Optional[int] = None) -> Tuple[str, np.ndarray]:
    """Exact payload bits and the restored cover from a .bin.

    Version 2 files carry the real start offset (and the search block size), which are used
    as stored.  Version 1 files (the reference's layout) store start_offset = 0
    (codec.py:903): the offset is re-derived by the block search on the restored plane 0,
    which needs the block size the file was encoded with -- search_block_size (default 16,
    main()'s value, codec.py:875); a different size decodes the wrong window."""
    md, blob, payload = container.parse_bin_file(filepath)
    s = md["s"]
    stego = _decompress(payload, md["codec"], md["height"], md["width"])
    bitmaps = container.split_bitmaps(blob, s)
    block = search_block_size or md.get("search_block_size") or 16
    offset = md["start_offset"] if md["version"] == 2 else None
    return api.decode_positional(stego, bitmaps, md, search_block_size=block,
                                 align_across_planes=bool(md["align_flag"]), start_offset=offset)


# ------------------------------------------------------------------ MED-PEE files
def encode_file_pee(image, payload, out_path: str, *, T=2, tmax: int = 16, maxval: Optional[int] = None,
                    codec: str = "raw", scheme: int = 1) -> Dict:
    """MED-PEE embed of one slice into a version-16 STGC file.  `image` is an array or a
    DICOM path; maxval defaults to the DICOM's full scale 2**BitsStored - 1 (4095 for the
    reference's 12-bit pe.dcm), else the dtype maximum.  T = 'auto' picks the smallest
    T <= tmax whose capacity holds the payload.  A payload beyond the capacity is truncated
    (status 1, 'L' = bits embedded); the file stays exactly reversible.  scheme 2: four
    sublattice passes (integer T; container scheme byte 2)."""
    from .pee import PeeCodec, lm_bits
    _require_gpu()
    torch = _torch()
    if isinstance(image, np.ndarray):
        img = image
    else:
        img, attrs = dicom.read_dicom(image)
        if maxval is None and attrs.get("bits_stored"):
            maxval = (1 << int(attrs["bits_stored"])) - 1
    if img.ndim != 2 or img.dtype not in (np.uint8, np.uint16):
        raise ValueError("A imagem deve ser 2D uint8 ou uint16.")
    h, w = img.shape
    bits = framing.to_bits(payload)
    pc = PeeCodec(1, h, w, dtype=str(img.dtype), T=T, tmax=tmax, maxval=maxval, scheme=scheme)
    enc = pc.embed(torch.from_numpy(np.ascontiguousarray(img)[None]).cuda(), [bits])
    if scheme == 2:
        prs = [pr[0] for pr in enc.pass_records()]
        blobs = [container.lm_blob(lm_bits(enc, 0, p)) if prs[p].end >= 0 else b"" for p in range(4)]
        embedded = enc.embedded()[0]
        status = 1 if embedded < len(bits) else 0
        stego = enc.stego.cpu().numpy()[0]
        hdr = container.create_pee2_header(codec, img.dtype.itemsize, w, h, pc.T, pc.maxval, embedded, status,
                                           [(r.L, r.end, r.status, len(b)) for r, b in zip(prs, blobs)])
        size = container.create_binary_file(out_path, hdr, _compress(stego, codec), b"".join(blobs))
        return {"path": out_path, "bytes": size, "T": pc.T, "L": embedded, "maxval": pc.maxval, "status": status,
                "scheme": 2, "passes": [{"L": r.L, "end": r.end, "status": r.status, "lm_count": r.lm_count}
                                        for r in prs], "stego": stego}
    r = enc.records()[0]
    embedded = min(len(bits), r.capacity) if r.status == 1 else len(bits)
    lmb = container.lm_blob(lm_bits(enc, 0)) if r.end >= 0 else b""
    stego = enc.stego.cpu().numpy()[0]
    hdr = container.create_pee_header(codec, img.dtype.itemsize, w, h, r.T, embedded, r.end, r.maxval, r.status,
                                      len(lmb))
    size = container.create_binary_file(out_path, hdr, _compress(stego, codec), lmb)
    return {"path": out_path, "bytes": size, "T": r.T, "L": embedded, "end": r.end, "maxval": r.maxval,
            "status": r.status, "lm_count": r.lm_count, "stego": stego}


def decode_bin_pee(filepath: str) -> Tuple[np.ndarray, np.ndarray]:
    """(payload bits as a 0/1 uint8 vector, restored cover) from a version-16 STGC file."""
    from .pee import PeeCodec
    _require_gpu()
    torch = _torch()
    with open(filepath, "rb") as f:
        raw = f.read()
    if container.pee_scheme(raw) == 2:
        return _decode_pee2(raw)
    md, blob, data = container.parse_pee_bytes(raw)
    h, w = md["height"], md["width"]
    stego = _decompress(data, md["codec"], h, w)
    if stego.dtype.itemsize != md["bytes"]:
        raise ValueError("stego pixel size does not match the MED-PEE header")
    pc = PeeCodec(1, h, w, dtype=str(stego.dtype), T=max(1, md["T"]), maxval=md["maxval"])
    lm = np.zeros(pc.lm_words * 64, dtype=bool)
    if md["end"] >= 0:
        lm[: md["end"] + 1] = container.lm_from_blob(blob, md["end"])
    lm_t = torch.from_numpy(np.packbits(lm, bitorder="little").view(np.int64).copy()).view(1, -1).cuda()
    m = _lib.PeeMeta()
    nc = (h // 2) * (w // 2)
    m.T, m.maxval, m.L, m.end = md["T"], md["maxval"], md["L"], md["end"]
    m.nc, m.ntiles = nc, (nc + 1023) // 1024
    m.tile_end = md["end"] // 1024 if md["end"] >= 0 else -1
    m.status, m.capacity, m.h, m.w = md["status"], md["L"], h, w
    meta = torch.frombuffer(bytearray(bytes(m)), dtype=torch.uint8).view(1, -1).cuda()
    pw = max(1, (md["L"] + 63) // 64)
    words, cover = pc.extract(torch.from_numpy(np.ascontiguousarray(stego)[None]).cuda(), meta, lm_t,
                              payload_words=pw)
    return framing.unpack_bits(words.cpu().numpy()[0], md["L"]), cover.cpu().numpy()[0]


def _decode_pee2(raw: bytes) -> Tuple[np.ndarray, np.ndarray]:
    """Scheme-2 file: the passes' records rebuilt from the header, then the reverse passes."""
    from .pee import PeeCodec, PeeEncoded, lattice_geometry
    torch = _torch()
    md, blobs, data = container.parse_pee2_bytes(raw)
    h, w = md["height"], md["width"]
    stego = _decompress(data, md["codec"], h, w)
    if stego.dtype.itemsize != md["bytes"]:
        raise ValueError("stego pixel size does not match the MED-PEE header")
    pc = PeeCodec(1, h, w, dtype=str(stego.dtype), T=max(1, md["T"]), maxval=md["maxval"], scheme=2)
    lm = np.zeros((4, 1, pc.lm_words * 64), dtype=bool)
    metas = bytearray()
    for p, ps in enumerate(md["passes"]):
        if ps["end"] >= 0:
            lm[p, 0, : ps["end"] + 1] = container.lm_from_blob(blobs[p], ps["end"])
        _y0, _x0, hc, wc = lattice_geometry(p, h, w)
        m = _lib.PeeMeta()
        nc = hc * wc
        m.T, m.maxval, m.L, m.end = md["T"], md["maxval"], ps["L"], ps["end"]
        m.nc, m.ntiles = nc, (nc + 1023) // 1024
        m.tile_end = ps["end"] // 1024 if ps["end"] >= 0 else -1
        m.status, m.capacity, m.h, m.w = ps["status"], ps["L"], h, w
        m.reserved[0] = p
        metas += bytes(m)
    meta_t = torch.frombuffer(metas, dtype=torch.uint8).view(4, 1, -1).cuda()
    lm_t = torch.from_numpy(np.packbits(lm, axis=-1, bitorder="little").view(np.int64).copy()).cuda()
    pw = max(1, (md["L"] + 63) // 64)
    enc = PeeEncoded(stego=torch.from_numpy(np.ascontiguousarray(stego)[None]).cuda(), lm=lm_t, meta=meta_t,
                     lengths=[md["L"]], payload_words=pw, config=pc.config, scheme=2)
    words, cover = pc.extract(enc.stego, enc.meta, enc.lm, payload_words=pw)
    return framing.unpack_bits(words.cpu().numpy()[0], md["L"]), cover.cpu().numpy()[0]
