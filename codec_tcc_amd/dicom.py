"""Minimal DICOM reader / writer for little-endian files.

pydicom is not available on this image; the path only needs the pixel matrix of
uncompressed slices (images/pe.dcm: Explicit VR LE, 12-bit in uint16; images/torax.dcm:
Implicit VR LE, uint8) and a Secondary-Capture writer equivalent to `create_dicom`
(codec.py:23-106).  The Deflated Explicit VR Little Endian transfer syntax -- the
reference's 'png' codec (codec.py:151-162 write, :203-206 read) -- is read and written
too: the dataset after the file-meta group is one raw deflate stream (zlib, wbits -15).
Encapsulated (JPEG-family) pixel data is refused with ValueError.
"""
from __future__ import annotations

import struct
import zlib
from typing import Dict, Optional, Tuple

import numpy as np

EXPLICIT_LE = "1.2.840.10008.1.2.1"
IMPLICIT_LE = "1.2.840.10008.1.2"
DEFLATED_LE = "1.2.840.10008.1.2.1.99"                      # codec.py:157
SECONDARY_CAPTURE = "1.2.840.10008.5.1.4.1.1.7"           # codec.py:42
_LONG_VR = {b"OB", b"OD", b"OF", b"OL", b"OV", b"OW", b"SQ", b"UC", b"UR", b"UT", b"UN", b"SV", b"UV"}
_UNDEF = 0xFFFFFFFF
_ITEM, _ITEM_END, _SEQ_END = (0xFFFE, 0xE000), (0xFFFE, 0xE00D), (0xFFFE, 0xE0DD)
_PIXEL = (0x7FE0, 0x0010)


class _Reader:
    def __init__(self, buf: bytes, explicit: bool):
        self.b = buf
        self.explicit = explicit

    def header(self, i: int, explicit: bool):
        g, e = struct.unpack_from("<HH", self.b, i)
        if (g, e) in (_ITEM, _ITEM_END, _SEQ_END):
            return (g, e), None, struct.unpack_from("<I", self.b, i + 4)[0], 8
        vr = self.b[i + 4:i + 6]
        if explicit and vr.isalpha() and vr.isupper():
            if vr in _LONG_VR:
                return (g, e), vr, struct.unpack_from("<I", self.b, i + 8)[0], 12
            return (g, e), vr, struct.unpack_from("<H", self.b, i + 6)[0], 8
        return (g, e), None, struct.unpack_from("<I", self.b, i + 4)[0], 8

    def skip_undefined(self, i: int, explicit: bool) -> int:
        """Skip a sequence of undefined length starting at i; return the offset after it."""
        while i < len(self.b):
            tag, _vr, ln, hl = self.header(i, explicit)
            i += hl
            if tag == _SEQ_END:
                return i
            if tag == _ITEM:
                if ln == _UNDEF:
                    i = self.elements(i, explicit, stop_at_item_end=True)[1]
                else:
                    i += ln
        raise ValueError("DICOM: unterminated sequence")

    def elements(self, i: int, explicit: bool, stop_at_item_end: bool = False, out: Optional[dict] = None):
        while i + 8 <= len(self.b):
            tag, vr, ln, hl = self.header(i, explicit)
            if stop_at_item_end and tag == _ITEM_END:
                return out, i + hl
            if tag == _PIXEL:
                if ln == _UNDEF:
                    raise ValueError("DICOM: encapsulated (compressed) pixel data is not supported")
                if out is not None:
                    out[tag] = (vr, i + hl, ln)
                return out, i + hl + ln
            if ln == _UNDEF:
                i = self.skip_undefined(i + hl, explicit)
                continue
            if out is not None:
                out[tag] = (vr, i + hl, ln)
            i += hl + ln
        return out, i


def _us(buf, ent):
    return struct.unpack_from("<H", buf, ent[1])[0]


def _str(buf, ent):
    return buf[ent[1]:ent[1] + ent[2]].rstrip(b"\x00 ").decode("ascii", errors="replace")


def read_dicom(src) -> Tuple[np.ndarray, Dict]:
    """Pixel array + a few attributes of an uncompressed LE DICOM file (path or bytes)."""
    buf = src if isinstance(src, (bytes, bytearray)) else open(src, "rb").read()
    buf = bytes(buf)
    if buf[128:132] != b"DICM":
        raise ValueError("DICOM: missing DICM preamble")
    meta = _Reader(buf, True)
    tags, i = {}, 132
    # file meta group (always explicit VR LE)
    while i + 8 <= len(buf) and struct.unpack_from("<H", buf, i)[0] == 0x0002:
        tag, vr, ln, hl = meta.header(i, True)
        tags[tag] = (vr, i + hl, ln)
        i += hl + ln
    ts = _str(buf, tags[(0x0002, 0x0010)]) if (0x0002, 0x0010) in tags else EXPLICIT_LE
    if ts not in (EXPLICIT_LE, IMPLICIT_LE, DEFLATED_LE):
        raise ValueError(f"DICOM: transfer syntax {ts} not supported (uncompressed or deflated little endian only)")
    if ts == DEFLATED_LE:   # the dataset is one raw deflate stream after the file meta
        buf = buf[:i] + zlib.decompress(buf[i:], -15)
    explicit = ts != IMPLICIT_LE
    ds = {}
    _Reader(buf, explicit).elements(i, explicit, out=ds)
    if _PIXEL not in ds:
        raise ValueError("DICOM: no pixel data")
    rows, cols = _us(buf, ds[(0x0028, 0x0010)]), _us(buf, ds[(0x0028, 0x0011)])
    alloc = _us(buf, ds[(0x0028, 0x0100)])
    stored = _us(buf, ds[(0x0028, 0x0101)]) if (0x0028, 0x0101) in ds else alloc
    signed = _us(buf, ds[(0x0028, 0x0103)]) if (0x0028, 0x0103) in ds else 0
    spp = _us(buf, ds[(0x0028, 0x0002)]) if (0x0028, 0x0002) in ds else 1
    frames = int(_str(buf, ds[(0x0028, 0x0008)]) or 1) if (0x0028, 0x0008) in ds else 1
    if alloc not in (8, 16) or spp != 1:
        raise ValueError("DICOM: only 8/16-bit single-sample images are supported")
    dt = np.dtype(("<i" if signed else "<u") + str(alloc // 8))
    _vr, off, ln = ds[_PIXEL]
    n = rows * cols * frames
    px = np.frombuffer(buf, dtype=dt, count=n, offset=off).copy()
    arr = px.reshape((frames, rows, cols) if frames > 1 else (rows, cols))
    return arr, {"rows": rows, "columns": cols, "bits_allocated": alloc, "bits_stored": stored,
                 "pixel_representation": signed, "frames": frames, "transfer_syntax": ts,
                 "pixel_offset": off, "pixel_length": ln}


# ------------------------------------------------------------------ writer
def _elem(g, e, vr: bytes, value: bytes) -> bytes:
    if len(value) % 2:
        value += b"\x00" if vr in (b"UI", b"OB") else b" "
    if vr in _LONG_VR:
        return struct.pack("<HH2sHI", g, e, vr, 0, len(value)) + value
    return struct.pack("<HH2sH", g, e, vr, len(value)) + value


def create_dicom_bytes(image: np.ndarray, *, sop_instance_uid: str = "1.2.826.0.1.3680043.10.1338.1",
                       study_uid: str = "1.2.826.0.1.3680043.10.1338.2", series_uid: str = "1.2.826.0.1.3680043.10.1338.3",
                       date: str = "20250101", time: str = "000000", transfer_syntax: str = EXPLICIT_LE,
                       level: int = -1) -> bytes:
    """Secondary Capture, Explicit VR LE -- the dataset create_dicom builds (codec.py:23-106),
    with caller-supplied UIDs/date so the output is deterministic.  transfer_syntax
    DEFLATED_LE deflates the dataset (the reference's 'png' codec, codec.py:151-162; zlib
    `level`); byte parity with pydicom's writer is unpinned (pydicom is absent here)."""
    if transfer_syntax not in (EXPLICIT_LE, DEFLATED_LE):
        raise ValueError(f"DICOM writer: transfer syntax {transfer_syntax} not supported")
    max_val = image.max()
    bits_stored = max(1, int(np.ceil(np.log2(float(max_val) + 1.0))))     # codec.py:27-32
    if image.ndim != 2:
        raise ValueError("A imagem deve ser 2D (grayscale).")               # codec.py:34
    if image.dtype not in (np.uint8, np.uint16):
        raise ValueError("A imagem deve ser uint8 ou uint16.")              # codec.py:36-37
    alloc = image.dtype.itemsize * 8
    rows, cols = image.shape
    us = lambda v: struct.pack("<H", v)                                      # noqa: E731
    ds = b"".join([
        _elem(0x0008, 0x0016, b"UI", SECONDARY_CAPTURE.encode()),
        _elem(0x0008, 0x0018, b"UI", sop_instance_uid.encode()),
        _elem(0x0008, 0x0020, b"DA", date.encode()),
        _elem(0x0008, 0x0023, b"DA", date.encode()),
        _elem(0x0008, 0x0030, b"TM", time.encode()),
        _elem(0x0008, 0x0033, b"TM", time.encode()),
        _elem(0x0008, 0x0060, b"CS", b"OT"),
        _elem(0x0010, 0x0010, b"PN", b"STEGO^"),
        _elem(0x0010, 0x0020, b"LO", b"123456"),
        _elem(0x0020, 0x000D, b"UI", study_uid.encode()),
        _elem(0x0020, 0x000E, b"UI", series_uid.encode()),
        _elem(0x0020, 0x0011, b"IS", b"1"),
        _elem(0x0020, 0x0013, b"IS", b"1"),
        _elem(0x0028, 0x0002, b"US", us(1)),
        _elem(0x0028, 0x0004, b"CS", b"MONOCHROME2"),
        _elem(0x0028, 0x0010, b"US", us(rows)),
        _elem(0x0028, 0x0011, b"US", us(cols)),
        _elem(0x0028, 0x0100, b"US", us(alloc)),
        _elem(0x0028, 0x0101, b"US", us(min(bits_stored, alloc))),
        _elem(0x0028, 0x0102, b"US", us(min(bits_stored, alloc) - 1)),
        _elem(0x0028, 0x0103, b"US", us(0)),
        _elem(0x0028, 0x1050, b"DS", str(int((int(image.max()) + int(image.min())) / 2)).encode()),
        _elem(0x0028, 0x1051, b"DS", str(int(image.max()) - int(image.min())).encode()),
        _elem(0x7FE0, 0x0010, b"OW" if alloc == 16 else b"OB", np.ascontiguousarray(image).astype("<u%d" % (alloc // 8)).tobytes()),
    ])
    meta_body = b"".join([
        _elem(0x0002, 0x0001, b"OB", b"\x00\x01"),
        _elem(0x0002, 0x0002, b"UI", SECONDARY_CAPTURE.encode()),
        _elem(0x0002, 0x0003, b"UI", sop_instance_uid.encode()),
        _elem(0x0002, 0x0010, b"UI", transfer_syntax.encode()),
        _elem(0x0002, 0x0012, b"UI", b"1.2.826.0.1.3680043.10.1338"),
    ])
    meta = _elem(0x0002, 0x0000, b"UL", struct.pack("<I", len(meta_body))) + meta_body
    if transfer_syntax == DEFLATED_LE:
        co = zlib.compressobj(level, zlib.DEFLATED, -15)
        ds = co.compress(ds) + co.flush()
        if len(ds) % 2:
            ds += b"\x00"   # even length (PS3.5 A.5)
    return b"\x00" * 128 + b"DICM" + meta + ds


def save_dicom(image: np.ndarray, path: str, **kw) -> int:
    """Write `image` as a Secondary-Capture file (save_dicom + create_dicom, codec.py:19-106)."""
    data = create_dicom_bytes(image, **kw)
    with open(path, "wb") as f:
        f.write(data)
    return len(data)
