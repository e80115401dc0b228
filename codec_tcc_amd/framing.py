"""Payload framing on the host: message bits and the per-plane segment plan.

These are the reference's two small host-side rules, restated for the product path:
  * message_to_bits           -- codec.py:239-240
  * distribute_message_segments -- codec.py:242-274 (quadratic weights, seed-42 shuffle,
    Python slice semantics for the chunking)
They cost microseconds per batch (the plan depends only on (T, s)), and feed the device
as a `codec_layout` table; no pixel work happens here.
"""
from __future__ import annotations

import functools
import random
from typing import Iterable, List, Sequence, Tuple

import numpy as np

from . import _lib


def message_to_bits(message: str) -> str:
    """codec.py:239-240: `{ord(c):08b}` per character (more than 8 bits for ord > 255)."""
    return "".join(format(ord(ch), "08b") for ch in message)


@functools.lru_cache(maxsize=None)
def plane_order(s: int) -> Tuple[int, ...]:
    """codec.py:262-264: `random.seed(42); random.shuffle(list(range(s)))`.  A private
    Random(42) has the same MT19937 state, so the global `random` state is not touched."""
    order = list(range(s))
    random.Random(42).shuffle(order)
    return tuple(order)


@functools.lru_cache(maxsize=4096)
def segment_plan(s: int, total_bits: int):
    """Return (sizes[s], perm[s], spans[s]) for a payload of `total_bits` over `s` planes.

    sizes: codec.py:251-259; perm: codec.py:262-264; spans[j] = (start, stop) of the j-th
    segment (taken for plane perm[j]) as `message_bits[bit_idx:bit_idx+size]` resolves it."""
    w = [(s - i) ** 2 for i in range(s)]
    tw = sum(w)
    sizes = [max(1, int((x / tw) * total_bits)) for x in w]
    extra = sum(sizes) - total_bits
    if extra != 0:
        k = sizes.index(max(sizes))
        sizes[k] -= extra
    perm = plane_order(s)
    spans = []
    at = 0
    for p in perm:
        a, b, _ = slice(at, at + sizes[p]).indices(total_bits)
        spans.append((a, max(a, b)))
        at += sizes[p]
    return tuple(sizes), perm, tuple(spans)


def distribute_message_segments(local_planes, message_bits: str):
    """Drop-in for codec.py:242-274: (segments, distributed_sizes, segment_indices)."""
    sizes, perm, spans = segment_plan(len(local_planes), len(message_bits))
    return [message_bits[a:b] for a, b in spans], list(sizes), list(perm)


@functools.lru_cache(maxsize=1024)
def _layout_rows(total_bits: int) -> bytes:
    rows = (_lib.Layout * 16)()
    for s in range(1, 17):
        sizes, perm, spans = segment_plan(s, total_bits)
        row = rows[s - 1]
        for j, p in enumerate(perm):
            row.perm[j] = p
            row.src[p] = spans[j][0]
            row.len[p] = spans[j][1] - spans[j][0]
        for p in range(s):
            row.sizes[p] = sizes[p]
    return bytes(rows)


def layout_table(lengths: Sequence[int]):
    """Per-batch layout table: one class per distinct payload length.

    Returns (table_bytes [n_classes*16 codec_layout], class_of_slice np.int32[B], n_classes)."""
    uniq = sorted(set(int(x) for x in lengths))
    idx = {t: i for i, t in enumerate(uniq)}
    table = b"".join(_layout_rows(t) for t in uniq)
    cls = np.asarray([idx[int(x)] for x in lengths], dtype=np.int32)
    return table, cls, len(uniq)


# ------------------------------------------------------------------ payload packing
def to_bits(payload) -> np.ndarray:
    """A payload as a uint8 0/1 vector in message order.

    str   -> message_to_bits (reference semantics, codec.py:239-240)
    bytes -> 8 bits per byte, MSB first (== message_to_bits of its latin-1 text)
    array -> taken as 0/1 bits already."""
    if isinstance(payload, str):
        bits = message_to_bits(payload)
        return np.frombuffer(bits.encode("ascii"), dtype=np.uint8) - ord("0")
    if isinstance(payload, (bytes, bytearray, memoryview)):
        return np.unpackbits(np.frombuffer(bytes(payload), dtype=np.uint8))
    arr = np.asarray(payload, dtype=np.uint8).ravel()
    if arr.size and arr.max() > 1:
        raise ValueError("bit payloads must contain only 0/1")
    return arr


def pack_bits(bit_vectors: Sequence[np.ndarray], words: int | None = None) -> Tuple[np.ndarray, List[int]]:
    """Pack 0/1 vectors LSB-first into uint64 words: [B, words] (int64 view), lengths."""
    lengths = [int(v.size) for v in bit_vectors]
    need = max([(n + 63) // 64 for n in lengths] + [1])
    words = max(words or 0, need)
    out = np.zeros((len(bit_vectors), words * 8), dtype=np.uint8)
    for i, v in enumerate(bit_vectors):
        if v.size:
            packed = np.packbits(v, bitorder="little")
            out[i, : packed.size] = packed
    return out.view(np.int64), lengths


def unpack_bits(words: np.ndarray, nbits: int) -> np.ndarray:
    """Inverse of pack_bits for one row."""
    raw = np.ascontiguousarray(words).view(np.uint8)
    return np.unpackbits(raw, bitorder="little")[:nbits]


def bits_to_str(bits: np.ndarray) -> str:
    return "".join("1" if b else "0" for b in bits.tolist())


def bits_to_bytes_msb(bits: np.ndarray) -> bytes:
    """codec.py:779-784: whole 8-bit chunks MSB-first; a trailing partial byte is dropped."""
    full = bits.size // 8 * 8
    return np.packbits(bits[:full]).tobytes() if full else b""
