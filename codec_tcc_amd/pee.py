"""MED-predictor prediction-error expansion (PEE) on the MI355X -- the algorithm the north
star names.  The reference contains no PEE code; the scheme is specified in
oracle/pee_cpu.py (parity unpinned) and summarised in include/codec_tcc.h.

    codec = PeeCodec(B, H, W, dtype="uint16", T=2)
    enc = codec.embed(covers, payloads)          # stego, location map, per-slice meta
    bits, cover = codec.decode(enc)

Scheme 2 (PeeCodec(..., scheme=2), oracle/pee_cpu.py "Scheme 2"): four sublattice passes on
the running image, about four times the capacity at one T; enc.meta / enc.lm then hold one
record / map per pass ([4, B, ...], pass-major).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib, framing
from .codec import _elem_bytes, _require_gpu, _stream, _torch


def lattice_geometry(lattice: int, H: int, W: int):
    """(y0, x0, hc, wc) of scheme 2's lattice p: candidate (i, j) is pixel (y0 + 2i, x0 + 2j),
    i < hc, j < wc (include/codec_tcc.h, codec_pee_multi_embed_pass)."""
    ry, rx = ((1, 1), (0, 0), (1, 0), (0, 1))[lattice]
    y0, x0 = (1 if ry else 2), (1 if rx else 2)
    return y0, x0, max(0, (H - y0 + 1) // 2), max(0, (W - x0 + 1) // 2)


@dataclass
class PeeEncoded:
    stego: object      # torch [B,H,W]
    lm: object         # torch.int64 [B, lm_words]: overflow location map, bit k = candidate k
    meta: object       # torch.uint8 [B, sizeof(codec_pee_meta)]
    lengths: List[int]
    payload_words: int
    config: dict = field(default_factory=dict)   # the PeeCodec's T / tmax / maxval (decode())
    scheme: int = 1                              # 2: four sublattice passes (meta / lm per pass)

    def records(self) -> List[_lib.PeeMeta]:
        """Scheme 1: one record per slice.  Scheme 2: 4 * B records, pass-major."""
        raw = self.meta.detach().cpu().contiguous().numpy().tobytes()
        n = len(raw) // _lib.PEE_META_BYTES
        return [_lib.PeeMeta.from_buffer_copy(raw, i * _lib.PEE_META_BYTES) for i in range(n)]

    def pass_records(self) -> List[List[_lib.PeeMeta]]:
        """Scheme 2: records[p][b] of pass p (scheme 1: one pass)."""
        recs = self.records()
        n = len(self.lengths)
        return [recs[i:i + n] for i in range(0, len(recs), n)]

    def embedded(self) -> List[int]:
        """Payload bits embedded per slice (scheme 2: the passes' sum)."""
        if self.scheme == 1:
            return [int(min(r.L, r.capacity)) if r.status == 1 else int(r.L) for r in self.records()]
        return [sum(int(pr[b].L) for pr in self.pass_records()) for b in range(len(self.lengths))]


class PeeCodec:
    def __init__(self, batch: int, height: int, width: int, dtype="uint16", *, T=2, tmax: int = 16,
                 maxval: Optional[int] = None, device=None, scheme: int = 1):
        """T: the expansion threshold for every slice, or "auto" -- capacity control: each
        slice gets the smallest T <= tmax whose capacity holds its payload
        (codec_pee_capacity, one extra read-only pass; meta.T records the choice).
        scheme: 1 = the (odd, odd) lattice in one pass; 2 = four sublattice passes
        (codec_pee_multi_embed_pass; integer T only)."""
        if scheme not in (1, 2):
            raise ValueError("scheme must be 1 or 2")
        if scheme == 2 and isinstance(T, str):
            raise ValueError("scheme 2 takes an integer T (capacity control is scheme 1's)")
        self.scheme = int(scheme)
        _require_gpu()
        torch = _torch()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        nbytes = 2 if "16" in str(dtype) else 1
        if str(dtype) not in ("uint16", "torch.uint16", "uint8", "torch.uint8"):
            raise ValueError("A imagem deve ser uint8 ou uint16.")
        vmax = 65535 if nbytes == 2 else 255
        self.B, self.H, self.W, self.bytes = int(batch), int(height), int(width), nbytes
        self.auto = isinstance(T, str)
        if self.auto and T != "auto":
            raise ValueError("T must be an integer >= 1 or 'auto'")
        self.T = 1 if self.auto else int(T)
        if not 1 <= int(tmax) <= 64:
            raise ValueError("tmax must be in 1..64")
        self.tmax = int(tmax)
        self.maxval = vmax if maxval is None else int(maxval)
        self.nc = (self.H // 2) * (self.W // 2)
        self.lm_words = max(1, (self.nc + 63) // 64)
        self.config = dict(method="pee", T="auto" if self.auto else self.T, tmax=self.tmax, maxval=self.maxval,
                           dtype="uint16" if nbytes == 2 else "uint8", scheme=self.scheme)
        P = self._params(1)
        ws = _lib.load().codec_pee_workspace_bytes(C.byref(P))
        if ws == 0:
            _lib.check(-1, "codec_pee_workspace_bytes")
        # zeroed by the reset below (codec_pee_reset: the whole workspace, the cumulative
        # look-back diagnostics included -- codec_pee_diag_offset)
        self.workspace = torch.empty(int(ws), dtype=torch.uint8, device=self.device)
        self.t_slices = torch.empty(self.B, dtype=torch.int32, device=self.device) if self.auto else None
        # register the fresh workspace with the library: an allocation at an address
        # an earlier workspace used would otherwise inherit that one's call-to-call state record
        self.reset()

    def reset(self):
        """Re-zero the workspace (codec_pee_reset, on the current stream): the state small
        out-of-place batches carry from call to call starts afresh, and the cumulative
        diagnostics read zero.  Called automatically after a failed call (include/codec_tcc.h,
        codec_pee_workspace_bytes: recovery rules)."""
        _lib.check(_lib.load().codec_pee_reset(C.byref(self._params(1)), self.workspace.data_ptr(),
                                               self.workspace.numel(), _stream()), "codec_pee_reset")

    def _guarded(self, fn, *args):
        """Run one workspace call; on any exception re-zero the workspace, then re-raise."""
        try:
            return fn(*args)
        except BaseException:
            try:
                self.reset()
            except Exception:   # the original error is the one to report
                pass
            raise

    def _params(self, payload_words: int) -> _lib.PeeParams:
        return _lib.PeeParams(B=self.B, H=self.H, W=self.W, bytes=self.bytes, T=self.T, maxval=self.maxval,
                              payload_words=int(payload_words), lm_words=self.lm_words)

    def pack_payloads(self, payloads):
        torch = _torch()
        bits = [framing.to_bits(p) for p in payloads]
        if len(bits) != self.B:
            raise ValueError("one payload per slice is required")
        packed, lengths = framing.pack_bits(bits)
        return (torch.from_numpy(packed).to(self.device), lengths,
                torch.tensor(lengths, dtype=torch.int32, device=self.device))

    def capacity(self, covers, tmax: Optional[int] = None):
        """int32 [B, tmax] device tensor: exact capacity of each slice at T = 1..tmax.
        Bounded by the candidate lattice: at most (H // 2) * (W // 2) bits per slice -- a
        quarter of the pixels; the other three quarters are the MED context, never modified."""
        torch = _torch()
        tmax = self.tmax if tmax is None else int(tmax)
        caps = torch.empty((self.B, tmax), dtype=torch.int32, device=self.device)
        self._guarded(lambda: _lib.check(_lib.load().codec_pee_capacity(
            C.byref(self._params(1)), covers.data_ptr(), tmax, None, caps.data_ptr(), None, self.workspace.data_ptr(),
            self.workspace.numel(), _stream()), "codec_pee_capacity"))
        return caps

    def embed(self, covers, payloads, *, stego=None, lm=None, meta=None, packed=None, check: bool = True) -> PeeEncoded:
        """cover -> stego + location map + per-slice meta.  check=True (default) reads the
        per-slice status back (one sync) and raises RuntimeError if an in-place look-back
        gave up (CODEC_PEE_ELOOKBACK: the slice is not a valid stego); check=False keeps
        the call asynchronous (benchmarks) -- inspect enc.records() afterwards."""
        torch = _torch()
        if tuple(covers.shape) != (self.B, self.H, self.W) or _elem_bytes(covers) != self.bytes:
            raise ValueError("covers do not match the codec's shape/dtype")
        words, lengths, lens_t = packed if packed is not None else self.pack_payloads(payloads)
        if stego is None:
            stego = torch.empty_like(covers)
        if self.scheme == 2:
            return self._embed_multi(covers, words, lengths, lens_t, stego, lm, meta, check)
        if lm is None:
            lm = torch.empty((self.B, self.lm_words), dtype=torch.int64, device=self.device)
        if meta is None:
            meta = torch.empty((self.B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=self.device)
        P = self._params(words.shape[1])
        lib = _lib.load()

        def launch():
            if self.auto:   # capacity control: per-slice T on the device (fused into the embed
                # launch where it runs slice-serial, else one read-only capacity pass first)
                _lib.check(lib.codec_pee_embed_auto(C.byref(P), covers.data_ptr(), stego.data_ptr(), words.data_ptr(),
                                                    lens_t.data_ptr(), self.tmax, self.t_slices.data_ptr(),
                                                    meta.data_ptr(), lm.data_ptr(), self.workspace.data_ptr(),
                                                    self.workspace.numel(), _stream()), "codec_pee_embed_auto")
            else:
                _lib.check(lib.codec_pee_embed_ts(C.byref(P), covers.data_ptr(), stego.data_ptr(), words.data_ptr(),
                                                  lens_t.data_ptr(), None, meta.data_ptr(), lm.data_ptr(),
                                                  self.workspace.data_ptr(), self.workspace.numel(), _stream()),
                           "codec_pee_embed")
        self._guarded(launch)
        enc = PeeEncoded(stego=stego, lm=lm, meta=meta, lengths=list(lengths), payload_words=int(words.shape[1]),
                         config=self.config)
        if check:
            recs = enc.records()
            if any(r.status not in (0, 1) for r in recs):   # not a capacity overflow: start clean
                self.reset()
            _raise_lookback(recs)
        return enc

    def _embed_multi(self, covers, words, lengths, lens_t, stego, lm, meta, check):
        """Scheme 2: passes 0..3 in one library call (codec_pee_multi_embed: one slice-serial
        launch after scheme 1's pass 0 on chip-filling batches, per-pass tile launches
        otherwise); pass 0 copies cover -> stego, the others run in place."""
        torch = _torch()
        if lm is None:
            lm = torch.empty((4, self.B, self.lm_words), dtype=torch.int64, device=self.device)
        if meta is None:
            meta = torch.empty((4, self.B, _lib.PEE_META_BYTES), dtype=torch.uint8, device=self.device)
        if tuple(lm.shape) != (4, self.B, self.lm_words) or tuple(meta.shape) != (4, self.B, _lib.PEE_META_BYTES):
            raise ValueError("scheme 2 takes lm [4, B, lm_words] and meta [4, B, PEE_META_BYTES]")
        if not (lm.is_contiguous() and meta.is_contiguous()):
            raise ValueError("scheme 2's lm and meta must be contiguous")
        P = self._params(words.shape[1])
        lib = _lib.load()
        self._guarded(lambda: _lib.check(lib.codec_pee_multi_embed(
            C.byref(P), covers.data_ptr(), stego.data_ptr(), words.data_ptr(), lens_t.data_ptr(), meta.data_ptr(),
            lm.data_ptr(), self.workspace.data_ptr(), self.workspace.numel(), _stream()), "codec_pee_multi_embed"))
        enc = PeeEncoded(stego=stego, lm=lm, meta=meta, lengths=list(lengths), payload_words=int(words.shape[1]),
                         config=self.config, scheme=2)
        if check:   # pass 0 in place runs scheme 1's look-back embed
            recs = enc.pass_records()[0]
            if any(r.status not in (0, 1) for r in recs):
                self.reset()
            _raise_lookback(recs)
        return enc

    def extract(self, stego, meta, lm, *, payload_words: int, cover=None, payload=None):
        torch = _torch()
        if cover is None:
            cover = torch.empty_like(stego)
        if payload is None:
            payload = torch.empty((self.B, int(payload_words)), dtype=torch.int64, device=self.device)
        if self.scheme == 2:
            return self._extract_multi(stego, meta, lm, payload_words, cover, payload)
        P = self._params(payload_words)
        self._guarded(lambda: _lib.check(_lib.load().codec_pee_extract(
            C.byref(P), stego.data_ptr(), meta.data_ptr(), lm.data_ptr(), cover.data_ptr(), payload.data_ptr(),
            self.workspace.data_ptr(), self.workspace.numel(), _stream()), "codec_pee_extract"))
        return payload, cover

    def _extract_multi(self, stego, meta, lm, payload_words, cover, payload):
        """Scheme 2: passes 3..0 in one library call (codec_pee_multi_extract; the first copies
        stego -> cover, the others run in place; payload written whole)."""
        if not (lm.is_contiguous() and meta.is_contiguous()):
            raise ValueError("scheme 2's lm and meta must be contiguous")
        P = self._params(payload_words)
        lib = _lib.load()
        self._guarded(lambda: _lib.check(lib.codec_pee_multi_extract(
            C.byref(P), stego.data_ptr(), meta.data_ptr(), lm.data_ptr(), cover.data_ptr(), payload.data_ptr(),
            self.workspace.data_ptr(), self.workspace.numel(), _stream()), "codec_pee_multi_extract"))
        return payload, cover

    def lookback_failed(self, payload_words: int = 1) -> bool:
        """True when the last in-place extract's look-back gave up (its payload is invalid)."""
        off = int(_lib.load().codec_pee_extract_flag_offset(C.byref(self._params(payload_words))))
        return bool(off) and int(self.workspace[off:off + 4].view(_torch().int32).item()) != 0

    def diagnostics(self, payload_words: int = 1) -> dict:
        """Cumulative look-back counters since construction (codec_pee_diag_offset)."""
        off = int(_lib.load().codec_pee_diag_offset(C.byref(self._params(payload_words))))
        v = self.workspace[off:off + 16].view(_torch().int32).cpu().tolist()
        return {"embed_fallback_chunks": v[0], "extract_fallback_chunks": v[1],
                "embed_unrecovered_chunks": v[2], "extract_unrecovered_chunks": v[3]}

    def repaired(self, payload_words: int = 1) -> int:
        """Chunks whose look-back fell back to counting predecessors from pixels (exact)."""
        d = self.diagnostics(payload_words)
        return d["embed_fallback_chunks"] + d["extract_fallback_chunks"]

    def decode(self, enc: PeeEncoded):
        """(list of 0/1 bit vectors, restored cover tensor); raises if a slice overflowed."""
        if enc.scheme != self.scheme:
            raise ValueError(f"a scheme-{enc.scheme} embedding given to a scheme-{self.scheme} codec")
        if self.scheme == 2:
            got = enc.embedded()
            short = [i for i, (g, n) in enumerate(zip(got, enc.lengths)) if g < n]
            if short:
                raise ValueError(f"payload exceeds PEE capacity in slices {short} (scheme 2, T={self.T})")
            words, cover = self.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
            host = words.cpu().numpy()   # the extract passes have no look-back (tile or slice-serial)
            return [framing.unpack_bits(host[i], enc.lengths[i]) for i in range(self.B)], cover
        recs = enc.records()
        _raise_lookback(recs)
        _raise_status(recs, f"T={'auto, tmax=%d' % self.tmax if self.auto else self.T}")
        words, cover = self.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
        host = words.cpu().numpy()
        if self.lookback_failed(enc.payload_words):
            self.reset()
            raise RuntimeError("codec_pee_extract: in-place cursor look-back timed out; the recovered "
                               "payload is invalid (the restored cover is exact)")
        return [framing.unpack_bits(host[i], enc.lengths[i]) for i in range(self.B)], cover


# one PeeCodec (and its zeroed workspace) per (shape, dtype, T, tmax, maxval, device); the
# least recently used one is dropped past _CODECS_MAX entries, so varied shapes do not keep
# GPU memory alive indefinitely (clear_codec_cache() drops them all)
_CODECS: "OrderedDict" = OrderedDict()
_CODECS_MAX = 8


def clear_codec_cache():
    """Drop every cached PeeCodec of encode()/decode() (frees their workspaces)."""
    _CODECS.clear()


def _codec_for(shape, dtype: str, *, T, tmax: int, maxval: Optional[int], scheme: int = 1) -> PeeCodec:
    torch = _torch()
    if maxval is None:
        maxval = 65535 if "16" in dtype else 255
    key = (tuple(shape), dtype, T, int(tmax), int(maxval), int(scheme), torch.cuda.current_device())
    c = _CODECS.get(key)
    if c is None:
        c = PeeCodec(*shape, dtype=dtype, T=T, tmax=tmax, maxval=maxval, scheme=scheme)
        _CODECS[key] = c
        while len(_CODECS) > _CODECS_MAX:
            _CODECS.popitem(last=False)
    else:
        _CODECS.move_to_end(key)
    return c


_STATUS_TEXT = {1: "payload exceeds PEE capacity", _lib.CODEC_PEE_ELOOKBACK: "in-place cursor look-back timed out"}


def _raise_status(recs, what: str):
    """ValueError for capacity overflows (status 1), RuntimeError naming any other code."""
    bad = {}
    for i, r in enumerate(recs):
        if r.status != 0:
            bad.setdefault(int(r.status), []).append(i)
    if not bad:
        return
    if set(bad) == {1}:
        raise ValueError(f"payload exceeds PEE capacity in slices {bad[1]} ({what})")
    text = "; ".join(f"status {c} ({_STATUS_TEXT.get(c, 'unknown status')}) in slices {v}" for c, v in sorted(bad.items()))
    raise RuntimeError(f"codec_pee: {text} ({what})")


def _config_from_records(enc: "PeeEncoded") -> dict:
    """The codec configuration of a PeeEncoded built without one (e.g. by hand): dtype from
    the stego tensor, maxval and T from the per-slice meta records."""
    recs = enc.records()
    if not recs:
        raise ValueError("PeeEncoded holds no slice records")
    dt = "uint16" if _elem_bytes(enc.stego) == 2 else "uint8"
    maxvals = {int(r.maxval) for r in recs}
    if len(maxvals) != 1:
        raise ValueError(f"slices were embedded with different maxval {sorted(maxvals)}; pass a config")
    ts = {int(r.T) for r in recs}
    T = ts.pop() if len(ts) == 1 else "auto"
    tmax = max(16, max(int(r.T) for r in recs))
    return dict(method="pee", T=T, tmax=min(tmax, 64), maxval=maxvals.pop(), dtype=dt)


def encode(covers, payloads: Sequence, *, T=2, tmax: int = 16, maxval: Optional[int] = None,
           scheme: int = 1) -> PeeEncoded:
    """MED-PEE embed of one payload per slice (the package's `encode(..., method="pee")`).
    covers: [B,H,W] / [H,W] uint8/uint16 torch tensor or numpy array; T: expansion threshold
    or "auto" (smallest T <= tmax whose capacity holds each slice's payload); maxval: the
    largest legal pixel value (e.g. 4095 for 12-bit DICOM; default the dtype's maximum);
    scheme 2: four sublattice passes (integer T).
    Raises ValueError when a payload exceeds its slice's capacity."""
    from .codec import _as_batch
    _require_gpu()
    covers = _as_batch(covers)
    if isinstance(payloads, (str, bytes, bytearray)):
        payloads = [payloads]
    dt = "uint16" if _elem_bytes(covers) == 2 else "uint8"
    codec = _codec_for(tuple(covers.shape), dt, T=T, tmax=tmax, maxval=maxval, scheme=scheme)
    enc = codec.embed(covers, payloads)
    if scheme == 2:
        short = [i for i, (g, n) in enumerate(zip(enc.embedded(), enc.lengths)) if g < n]
        if short:
            raise ValueError(f"payload exceeds PEE capacity in slices {short} (scheme 2, T={T})")
    else:
        _raise_status(enc.records(), f"T={T}, tmax={tmax}")
    return enc


def decode(enc: PeeEncoded, *, restore: bool = True):
    """Exact extraction: (payload_bit_lists, cover) like the LSB decode() -- payload_bit_lists[b]
    is a numpy 0/1 vector of slice b's embedded bits, cover the restored [B,H,W] tensor
    (None with restore=False)."""
    _require_gpu()
    cfg = enc.config or _config_from_records(enc)
    codec = _codec_for(tuple(enc.stego.shape), cfg.get("dtype", "uint16"), T=cfg.get("T", 2),
                       tmax=cfg.get("tmax", 16), maxval=cfg.get("maxval"), scheme=int(getattr(enc, "scheme", 1)))
    bits, cover = codec.decode(enc)
    return bits, (cover if restore else None)


def _raise_lookback(recs):
    lost = [i for i, r in enumerate(recs) if r.status == _lib.CODEC_PEE_ELOOKBACK]
    if lost:
        raise RuntimeError(f"codec_pee_embed: in-place cursor look-back timed out in slices {lost}; "
                           "their pixels are not a valid stego")


def lm_bits(enc: PeeEncoded, b: int, p: int = 0) -> np.ndarray:
    """Location map of slice b (scheme 2: of pass p) as a bool vector over candidates 0..end."""
    if enc.scheme == 2:
        r = enc.pass_records()[p][b]
        raw = enc.lm[p, b].cpu().numpy().view(np.uint8)
    else:
        r = enc.records()[b]
        raw = enc.lm[b].cpu().numpy().view(np.uint8)
    return np.unpackbits(raw, bitorder="little")[: r.end + 1].astype(bool)
