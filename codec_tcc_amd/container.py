"""The ".bin" container ("STGC") either side of the pixel path.

Version 1 is byte-compatible with the reference (codec.py:601-750):

    b"STGC" | >I header_length | header | zlib(dense bitmaps) | compressed stego
    header v1 = >BBBBHHH (version=1, codec_id, s, align, width, height, start_offset)
                + s*>H segments_lengths + s*>B segment_indices + >I bitmaps_blob_size

Its 16-bit fields overflow at 2048^2 (struct.error) and main() writes
start_offset=0 (codec.py:903).  Version 2 (this build's extension) widens width, height,
start_offset and segments_lengths to 32 bits (segments_lengths signed: T < s plans have
negative sizes) and stores the real offset:

    header v2 = >BBBBIIi (version=2, codec_id, s, align, width, height, start_offset)
                + s*>i segments_lengths + s*>B segment_indices + >I bitmaps_blob_size

Stego payload codecs: the reference's ids (png 1, j2k 2, jls 3, jxl 4) are kept; id 0
("raw", unknown to the reference) stores the stego pixels little-endian, uncompressed.
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import Dict, List, Sequence, Tuple

import numpy as np

MAGIC = b"STGC"
CODEC_IDS = {"png": 1, "j2k": 2, "jls": 3, "jxl": 4}     # codec.py:616
CODEC_NAMES = {1: "png", 2: "j2k", 3: "jls", 4: "jxl"}   # codec.py:693


def create_header(codec: str, s: int, segments_lengths: Sequence[int], segments_indices: Sequence[int],
                  bitmaps_blob_size: int, width: int, height: int, start_offset: int,
                  align_across_planes: bool, version: int = 1) -> bytes:
    """codec.py:601-656 (version 1, identical bytes; raises struct.error where it does)."""
    cid = CODEC_IDS.get(codec.lower(), 0)
    flag = 1 if align_across_planes else 0
    if version == 1:
        fmt = ">BBBBHHH" + f"{s}H" + f"{s}B" + "I"
    elif version == 2:
        fmt = ">BBBBIIi" + f"{s}i" + f"{s}B" + "I"
    else:
        raise ValueError(f"unknown container version {version}")
    return struct.pack(fmt, version, cid, s, flag, width, height, start_offset,
                       *list(segments_lengths), *list(segments_indices), bitmaps_blob_size)


def create_binary_file(filename: str, header_bytes: bytes, stego_compressed: bytes, bitmaps_bytes: bytes) -> int:
    """codec.py:658-670: STGC + >I len + header + bitmap blob + stego; returns the file size."""
    with open(filename, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack(">I", len(header_bytes)))
        f.write(header_bytes)
        f.write(bitmaps_bytes)
        f.write(stego_compressed)
    return os.path.getsize(filename)


def parse_bin_bytes(data: bytes) -> Tuple[Dict, bytes, bytes]:
    if data[:4] != MAGIC:
        raise ValueError("Arquivo inválido ou com assinatura incorreta.")   # codec.py:698
    (hlen,) = struct.unpack(">I", data[4:8])
    hdr = data[8:8 + hlen]
    version = hdr[0]
    base = ">BBBBHHH" if version == 1 else ">BBBBIIi"
    nb = struct.calcsize(base)
    version, cid, s, flag, width, height, start = struct.unpack(base, hdr[:nb])
    lf = f">{s}H" if version == 1 else f">{s}i"
    nl = struct.calcsize(lf)
    lens = list(struct.unpack(lf, hdr[nb:nb + nl]))
    idx = list(struct.unpack(f">{s}B", hdr[nb + nl:nb + nl + s]))
    (blob_size,) = struct.unpack(">I", hdr[nb + nl + s:nb + nl + s + 4])
    body = data[8 + hlen:]
    md = {"version": version, "codec": CODEC_NAMES.get(cid, "unknown"), "s": s, "align_flag": flag,
          "width": width, "height": height, "start_offset": start, "segments_lengths": lens,
          "segments_indices": idx}
    return md, body[:blob_size], body[blob_size:]


def parse_bin_file(filepath: str) -> Tuple[Dict, bytes, bytes]:
    """codec.py:689-750 -> (metadata, bitmaps_blob, stego_bytes)."""
    with open(filepath, "rb") as f:
        return parse_bin_bytes(f.read())


def bitmaps_blob(dense: np.ndarray) -> bytes:
    """zlib of the stacked s x H x W uint8 bitmaps (codec.py:888-889)."""
    return zlib.compress(np.ascontiguousarray(dense, dtype=np.uint8).tobytes())


def split_bitmaps(blob: bytes, s: int) -> List[np.ndarray]:
    """codec.py:820-821: zlib.decompress + np.split into s flat planes."""
    return np.split(np.frombuffer(zlib.decompress(blob), dtype=np.uint8), s)


def encode_stego_raw(stego: np.ndarray) -> bytes:
    return np.ascontiguousarray(stego).astype(stego.dtype.newbyteorder("<"), copy=False).tobytes()


def decode_stego_raw(data: bytes, height: int, width: int) -> np.ndarray:
    npx = height * width
    itemsize = len(data) // npx if npx else 0
    if itemsize not in (1, 2) or itemsize * npx != len(data):
        raise ValueError("raw stego payload does not match the header's width x height")
    return np.frombuffer(data, dtype="<u2" if itemsize == 2 else np.uint8).reshape(height, width).astype(
        np.uint16 if itemsize == 2 else np.uint8)
