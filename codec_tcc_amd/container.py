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
                [+ >H search_block_size]   (optional; 0 / absent = unknown)

MED-PEE files (this build's scheme; the reference has no PEE format) use
the same magic and framing with version 16:

    header pee = >BBBB (version=16, codec_id, bytes per pixel, scheme byte 0)
                 + >II (width, height) + >iiiii (T, L = embedded bits, end, maxval, status)
                 + >I lm_blob_size
    body       = zlib(location-map bits of candidates 0..end, LSB-first) | compressed stego

MED-PEE scheme 2 (four sublattice passes, oracle/pee_cpu.py) sets the scheme byte to 2:

    header pee2 = >BBBB (version=16, codec_id, bytes per pixel, 2)
                  + >II (width, height) + >iiii (T, maxval, L = embedded bits, status)
                  + 4 x >iiiI (L_p, end_p, status_p, lm_blob_size_p)
    body        = the 4 passes' zlib location maps in pass order | compressed stego

so a reader of scheme-1 files (scheme byte 0) refuses scheme-2 files instead of misreading.

Stego payload codecs: the reference's ids (png 1, j2k 2, jls 3, jxl 4) are kept; id 0
("raw", unknown to the reference) stores the stego pixels little-endian, uncompressed.
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

MAGIC = b"STGC"
PEE_VERSION = 16
CODEC_IDS = {"png": 1, "j2k": 2, "jls": 3, "jxl": 4}     # codec.py:616
CODEC_NAMES = {1: "png", 2: "j2k", 3: "jls", 4: "jxl"}   # codec.py:693


def create_header(codec: str, s: int, segments_lengths: Sequence[int], segments_indices: Sequence[int],
                  bitmaps_blob_size: int, width: int, height: int, start_offset: int,
                  align_across_planes: bool, version: int = 1, search_block_size: Optional[int] = None) -> bytes:
    """codec.py:601-656 (version 1, identical bytes; raises struct.error where it does).
    Version 2 may also record the block size of the start-offset search."""
    cid = CODEC_IDS.get(codec.lower(), 0)
    flag = 1 if align_across_planes else 0
    if version == 1:
        fmt = ">BBBBHHH" + f"{s}H" + f"{s}B" + "I"
    elif version == 2:
        fmt = ">BBBBIIi" + f"{s}i" + f"{s}B" + "I"
    else:
        raise ValueError(f"unknown container version {version}")
    hdr = struct.pack(fmt, version, cid, s, flag, width, height, start_offset,
                      *list(segments_lengths), *list(segments_indices), bitmaps_blob_size)
    if version == 2 and search_block_size is not None:
        hdr += struct.pack(">H", int(search_block_size))
    return hdr


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
    if version == PEE_VERSION:
        raise ValueError("a MED-PEE container (version 16): use parse_pee_bytes / decode_bin_pee")
    base = ">BBBBHHH" if version == 1 else ">BBBBIIi"
    nb = struct.calcsize(base)
    version, cid, s, flag, width, height, start = struct.unpack(base, hdr[:nb])
    lf = f">{s}H" if version == 1 else f">{s}i"
    nl = struct.calcsize(lf)
    lens = list(struct.unpack(lf, hdr[nb:nb + nl]))
    idx = list(struct.unpack(f">{s}B", hdr[nb + nl:nb + nl + s]))
    (blob_size,) = struct.unpack(">I", hdr[nb + nl + s:nb + nl + s + 4])
    rest = hdr[nb + nl + s + 4:]
    body = data[8 + hlen:]
    md = {"version": version, "codec": CODEC_NAMES.get(cid, "unknown"), "s": s, "align_flag": flag,
          "width": width, "height": height, "start_offset": start, "segments_lengths": lens,
          "segments_indices": idx}
    if version == 2 and len(rest) >= 2:
        md["search_block_size"] = struct.unpack(">H", rest[:2])[0] or None
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


# ------------------------------------------------------------------ MED-PEE container
_PEE_FMT = ">BBBBIIiiiiiI"


def create_pee_header(codec: str, bytes_per_px: int, width: int, height: int, T: int, L: int, end: int,
                      maxval: int, status: int, lm_blob_size: int) -> bytes:
    return struct.pack(_PEE_FMT, PEE_VERSION, CODEC_IDS.get(codec.lower(), 0), int(bytes_per_px), 0, width, height,
                       int(T), int(L), int(end), int(maxval), int(status), int(lm_blob_size))


def lm_blob(lm_bits: np.ndarray) -> bytes:
    """zlib of the location-map bits (candidates 0..end), packed LSB-first."""
    return zlib.compress(np.packbits(np.asarray(lm_bits, dtype=np.uint8), bitorder="little").tobytes())


def lm_from_blob(blob: bytes, end: int) -> np.ndarray:
    raw = np.frombuffer(zlib.decompress(blob), dtype=np.uint8)
    return np.unpackbits(raw, bitorder="little")[: end + 1].astype(bool)


_PEE2_FMT = ">BBBBIIiiii"
_PEE2_PASS = ">iiiI"
PEE_SCHEME2 = 2


def create_pee2_header(codec: str, bytes_per_px: int, width: int, height: int, T: int, maxval: int, L: int,
                       status: int, passes: Sequence[Tuple[int, int, int, int]]) -> bytes:
    """Scheme-2 header; passes = 4 x (L_p, end_p, status_p, lm_blob_size_p)."""
    if len(passes) != 4:
        raise ValueError("scheme 2 has four passes")
    hdr = struct.pack(_PEE2_FMT, PEE_VERSION, CODEC_IDS.get(codec.lower(), 0), int(bytes_per_px), PEE_SCHEME2,
                      width, height, int(T), int(maxval), int(L), int(status))
    return hdr + b"".join(struct.pack(_PEE2_PASS, int(a), int(b), int(c), int(d)) for a, b, c, d in passes)


def pee_scheme(data: bytes) -> int:
    """1 or 2: the MED-PEE scheme of a version-16 STGC file (its scheme byte)."""
    if data[:4] != MAGIC:
        raise ValueError("Arquivo inválido ou com assinatura incorreta.")   # codec.py:698
    (hlen,) = struct.unpack(">I", data[4:8])
    hdr = data[8:8 + hlen]
    if len(hdr) < 4 or hdr[0] != PEE_VERSION:
        raise ValueError("not a MED-PEE container (version 16)")
    if hdr[3] not in (0, PEE_SCHEME2):
        raise ValueError(f"unknown MED-PEE scheme byte {hdr[3]}")
    return 2 if hdr[3] == PEE_SCHEME2 else 1


def parse_pee2_bytes(data: bytes) -> Tuple[Dict, List[bytes], bytes]:
    """A scheme-2 version-16 STGC file -> (side information with 'passes', 4 lm blobs, stego bytes)."""
    if pee_scheme(data) != 2:
        raise ValueError("not a scheme-2 MED-PEE container")
    (hlen,) = struct.unpack(">I", data[4:8])
    hdr = data[8:8 + hlen]
    n0 = struct.calcsize(_PEE2_FMT)
    (_v, cid, bpp, _s, width, height, T, maxval, L, status) = struct.unpack(_PEE2_FMT, hdr[:n0])
    passes, blobs, body, pos = [], [], data[8 + hlen:], 0
    for p in range(4):
        Lp, endp, stp, nb = struct.unpack(_PEE2_PASS, hdr[n0 + 16 * p: n0 + 16 * (p + 1)])
        passes.append({"L": Lp, "end": endp, "status": stp})
        blobs.append(body[pos:pos + nb])
        pos += nb
    md = {"version": PEE_VERSION, "scheme": 2, "codec": CODEC_NAMES.get(cid, "raw" if cid == 0 else "unknown"),
          "bytes": bpp, "width": width, "height": height, "T": T, "maxval": maxval, "L": L, "status": status,
          "passes": passes}
    return md, blobs, body[pos:]


def parse_pee_bytes(data: bytes) -> Tuple[Dict, bytes, bytes]:
    """A version-16 STGC file of scheme 1 -> (side information, lm_blob, stego bytes)."""
    if pee_scheme(data) != 1:
        raise ValueError("a scheme-2 MED-PEE container: use parse_pee2_bytes")
    (hlen,) = struct.unpack(">I", data[4:8])
    hdr = data[8:8 + hlen]
    (_v, cid, bpp, _r, width, height, T, L, end, maxval, status, blob_size) = struct.unpack(
        _PEE_FMT, hdr[:struct.calcsize(_PEE_FMT)])
    body = data[8 + hlen:]
    md = {"version": PEE_VERSION, "codec": CODEC_NAMES.get(cid, "raw" if cid == 0 else "unknown"),
          "bytes": bpp, "width": width, "height": height, "T": T, "L": L, "end": end, "maxval": maxval,
          "status": status}
    return md, body[:blob_size], body[blob_size:]
