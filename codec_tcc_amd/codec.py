"""Batched host orchestration of the HIP path: encode() / decode() on [B,H,W] tensors.

Pixels stay in HBM as torch tensors; every pixel operation is a HIP kernel reached through
the C ABI (include/codec_tcc.h).  The host only frames payloads (framing.py), builds the
segment-layout table, and owns buffers.  There is no CPU fallback: without a GPU or
without libcodec_hip.so every call raises.

Reference correspondence (wesleyfn/codec-tcc, src/codec.py):
  encode  = adaptive_modalities_decomposition (:561) + lsb_embed_block_then_multiplane
            (:412, search_block_size=16 as main() uses at :874-876) + merge_modalities (:215)
  decode  = positional recovery of the payload + cover restore
  decode_ref_compat = extract_local_planes (:789) + decode_message (:752), bit-exact
            with the reference's (lossy) output string
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib, framing

_TORCH = None


def _torch():
    global _TORCH
    if _TORCH is None:
        import torch
        _TORCH = torch
    return _TORCH


def _require_gpu():
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("codec_tcc_amd needs an MI355X (ROCm) device: no GPU visible and no CPU fallback")
    _lib.load()


def _stream():
    return _torch().cuda.current_stream().cuda_stream


def _pix_dtype(nbytes: int):
    torch = _torch()
    return torch.uint16 if nbytes == 2 else torch.uint8


def _elem_bytes(t) -> int:
    torch = _torch()
    if t.dtype == torch.uint16 or t.dtype == torch.int16:
        return 2
    if t.dtype == torch.uint8:
        return 1
    raise TypeError(f"pixels must be uint8 or uint16, got {t.dtype}")


def _padded_empty(shape, dtype, device):
    """Tensor whose storage has >= 16 spare bytes (atomic 32-bit word writes at the end)."""
    torch = _torch()
    n = int(np.prod(shape))
    esz = torch.empty((), dtype=dtype).element_size()
    flat = torch.empty(n + max(1, 16 // esz), dtype=dtype, device=device)
    return flat[:n].view(*shape)


# ------------------------------------------------------------------ numpy log2 table
_LUT = {}


def log2_table(npix: int, device):
    """lut[c-1] = numpy.log2(c / npix), c = 1..npix, on `device` (cached).

    These are exactly the values calculate_entropy / calculate_mutual_information
    compute elementwise (`np.log2(counts[counts>0] / size)`, codec.py:498-501,531,543,550):
    numpy's log2 on this host's CPU.  The device multiplies and sums them in numpy's
    order, so the plane count s is decided bit-exactly as the reference decides it."""
    torch = _torch()
    key = (str(device), int(npix))
    t = _LUT.get(key)
    if t is None:
        lut = np.log2(np.arange(1, npix + 1, dtype=np.int64) / npix)
        t = torch.from_numpy(lut).to(device)
        _LUT[key] = t
    return t


# ------------------------------------------------------------------ payloads
@dataclass
class Payloads:
    """Device-resident packed payloads plus the per-batch segment-layout table."""
    words: object              # torch.int64 [B, payload_words], LSB-first bit packing
    lengths: List[int]         # payload length T (bits) per slice
    table: object              # torch.uint8 [n_classes*16*sizeof(codec_layout)]
    classes: object            # torch.int32 [B]
    n_classes: int
    map_words: int             # words needed for any location map of this batch

    @property
    def payload_words(self) -> int:
        return int(self.words.shape[1])


def make_payloads(payloads, device) -> Payloads:
    """Pack per-slice payloads (str / bytes / 0-1 arrays) and upload them."""
    torch = _torch()
    bits = [framing.to_bits(p) for p in payloads]
    lengths = [int(b.size) for b in bits]
    table, cls, ncls = framing.layout_table(lengths)
    # every embedded bit has one location-map bit and one recovered-payload bit; with
    # degenerate plans (T < s) the segments may overlap, so size by the plans themselves
    maxbits = max([1] + lengths)
    for t in set(lengths):
        for s in range(1, 17):
            _sz, _perm, spans = framing.segment_plan(s, t)
            maxbits = max(maxbits, sum(b - a for a, b in spans))
    map_words = (maxbits + 63) // 64
    packed, _ = framing.pack_bits(bits, words=map_words)
    return Payloads(
        words=torch.from_numpy(packed).to(device),
        lengths=lengths,
        table=torch.frombuffer(bytearray(table), dtype=torch.uint8).to(device),
        classes=torch.from_numpy(cls).to(device),
        n_classes=ncls,
        map_words=map_words,
    )


# ------------------------------------------------------------------ results
def meta_records(meta) -> List[_lib.SliceMeta]:
    """Device meta tensor [B, sizeof(codec_slice_meta)] -> list of ctypes records."""
    raw = meta.detach().to("cpu").contiguous().numpy().tobytes()
    n = len(raw) // _lib.META_BYTES
    return [_lib.SliceMeta.from_buffer_copy(raw, i * _lib.META_BYTES) for i in range(n)]


def meta_dict(m: _lib.SliceMeta) -> dict:
    s = m.s
    return {
        "s": s,
        "start_offset": m.start_offset,
        "total_used": m.total_used,
        "segment_indices": [m.perm[j] for j in range(s)],
        "segments_lengths": [m.sizes[p] for p in range(s)],
        "n": [m.n[p] for p in range(s)],
        "off": [m.off[p] for p in range(s)],
        "flags": m.flags,
        "entropy": m.entropy,
        "mi": [m.mi[i] for i in range(m.nbits)],
        "status": m.status,
    }


def check_status(recs, what: str = "codec_encode"):
    """Raise when a slice's meta.status says its decision may differ from the reference's:
    1 = the log2 table does not cover the slice (no exact entropy), 2 = a split decision's
    plane workgroup never published (CODEC_FLAG_DECIDE_TIMEOUT: that plane's MI is unknown,
    so `s` can differ).  The round trip of such a slice is still exact (decode reads s from
    the meta), which is why a caller has to look."""
    bad = [(i, r.status) for i, r in enumerate(recs) if r.status != 0]
    if bad:
        why = {1: "log2 table too short", 2: "split decision timed out"}
        raise RuntimeError(f"{what}: slices without the reference's decision: "
                           + ", ".join(f"{i} (status {s}: {why.get(s, 'unknown')})" for i, s in bad[:8])
                           + (" ..." if len(bad) > 8 else ""))


@dataclass
class Encoded:
    stego: object      # torch [B,H,W]
    maps: object       # torch.int64 [B, map_words]  packed location maps (segment order)
    meta: object       # torch.uint8 [B, sizeof(codec_slice_meta)]
    payloads: Payloads
    config: dict = field(default_factory=dict)

    def records(self):
        return meta_records(self.meta)


# ------------------------------------------------------------------ the codec
class Codec:
    """A configured encoder/decoder for batches of one shape and dtype.

    Buffers that do not depend on the data (workspace, log2 table) are allocated once,
    so repeated calls launch kernels only (graph-capturable, no host syncs)."""

    def __init__(self, batch: int, height: int, width: int, dtype="uint16", *, beta: float = 0.4,
                 block: int = 16, align: bool = False, mode: str = "hybrid", nbits: Optional[int] = None,
                 fixed_s: int = 0, fixed_offset: int = -1, all_mi: bool = False, device=None):
        _require_gpu()
        torch = _torch()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        in_bytes = 2 if str(dtype) in ("uint16", "torch.uint16", "int16", "torch.int16") else 1
        if str(dtype) not in ("uint16", "torch.uint16", "int16", "torch.int16", "uint8", "torch.uint8"):
            raise ValueError("A imagem deve ser uint8 ou uint16.")   # codec.py:36-37
        nb = in_bytes * 8 if nbits is None else int(nbits)
        if not 1 <= nb <= 16:
            raise ValueError("nbits must be in 1..16")
        if block < 1:
            raise ValueError("search_block_size must be >= 1")
        if mode not in ("hybrid", "multi"):
            raise ValueError("mode must be 'hybrid' or 'multi'")
        self.B, self.H, self.W = int(batch), int(height), int(width)
        self.in_bytes = in_bytes
        self.out_bytes = 2 if nb > 8 else 1          # merge_modalities dtype rule, codec.py:221
        self.P = _lib.Params(
            B=self.B, H=self.H, W=self.W, in_bytes=in_bytes, out_bytes=self.out_bytes, nbits=nb,
            block=int(block), align=int(bool(align)),
            mode=_lib.MODE_HYBRID if mode == "hybrid" else _lib.MODE_MULTI,
            fixed_s=int(fixed_s), fixed_offset=int(fixed_offset), all_mi=int(bool(all_mi)),
            payload_words=1, map_words=1, n_classes=1, reserved=0, beta=float(beta))
        self.config = dict(beta=float(beta), block=int(block), align=bool(align), mode=mode, nbits=nb)
        lib = _lib.load()
        ws = lib.codec_workspace_bytes(C.byref(self.P))
        if ws == 0:
            _lib.check(-1, "codec_workspace_bytes")
        # zero once: codec_plan expects clean histogram words and leaves them clean
        self.workspace = torch.zeros(int(ws), dtype=torch.uint8, device=self.device)
        self.lut = log2_table(self.H * self.W, self.device)

    # -- helpers
    def _params(self, pl: Optional[Payloads] = None, **over) -> _lib.Params:
        P = _lib.Params.from_buffer_copy(bytes(self.P))
        if pl is not None:
            P.payload_words = pl.payload_words
            P.map_words = pl.map_words
            P.n_classes = pl.n_classes
        for k, v in over.items():
            setattr(P, k, v)
        return P

    def _check_pixels(self, t, nbytes):
        torch = _torch()
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise TypeError("pixels must be a CUDA/ROCm torch tensor")
        if tuple(t.shape) != (self.B, self.H, self.W):
            raise ValueError(f"expected shape {(self.B, self.H, self.W)}, got {tuple(t.shape)}")
        if _elem_bytes(t) != nbytes:
            raise TypeError(f"expected {nbytes}-byte pixels, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError("pixel tensor must be contiguous")

    # -- encode: codec_encode (= codec_plan + codec_embed, fused when the dtypes allow)
    def encode(self, covers, payloads, *, stego=None, maps=None, meta=None, check: bool = True) -> Encoded:
        """check=True (default) reads the per-slice status back (one sync) and raises when a
        slice's decision is not the reference's (check_status); check=False keeps the call
        asynchronous (benchmarks, graph capture) -- inspect enc.records() afterwards."""
        torch = _torch()
        self._check_pixels(covers, self.in_bytes)
        pl = payloads if isinstance(payloads, Payloads) else make_payloads(payloads, self.device)
        if len(pl.lengths) != self.B:
            raise ValueError("one payload per slice is required")
        P = self._params(pl)
        if stego is None:
            stego = _padded_empty((self.B, self.H, self.W), _pix_dtype(self.out_bytes), self.device)
        if maps is None:
            maps = torch.empty((self.B, pl.map_words), dtype=torch.int64, device=self.device)
        if meta is None:
            meta = torch.empty((self.B, _lib.META_BYTES), dtype=torch.uint8, device=self.device)
        lib = _lib.load()
        st = _stream()
        _lib.check(lib.codec_encode(C.byref(P), covers.data_ptr(), stego.data_ptr(), self.lut.data_ptr(),
                                    self.lut.numel(), pl.table.data_ptr(), pl.classes.data_ptr(),
                                    meta.data_ptr(), self.workspace.data_ptr(), self.workspace.numel(),
                                    pl.words.data_ptr(), maps.data_ptr(), st), "codec_encode")
        if check:
            check_status(meta_records(meta), "codec_encode")
        return Encoded(stego=stego, maps=maps, meta=meta, payloads=pl, config=dict(self.config))

    # -- plan only (decomposition + offset, no payload writes)
    def plan(self, covers, payloads, *, stego=None, meta=None, check: bool = True):
        torch = _torch()
        self._check_pixels(covers, self.in_bytes)
        pl = payloads if isinstance(payloads, Payloads) else make_payloads(payloads, self.device)
        P = self._params(pl)
        if meta is None:
            meta = torch.empty((self.B, _lib.META_BYTES), dtype=torch.uint8, device=self.device)
        lib = _lib.load()
        _lib.check(lib.codec_plan(C.byref(P), covers.data_ptr(), None if stego is None else stego.data_ptr(),
                                  self.lut.data_ptr(), self.lut.numel(), pl.table.data_ptr(),
                                  pl.classes.data_ptr(), meta.data_ptr(), self.workspace.data_ptr(),
                                  self.workspace.numel(), _stream()), "codec_plan")
        if check:
            check_status(meta_records(meta), "codec_plan")
        return meta

    # -- decode: payload recovery + cover restore
    def decode(self, stego, maps, meta, *, payload_words: int, map_words: int, restore: bool = True,
               cover=None, payload=None):
        torch = _torch()
        self._check_pixels(stego, self.out_bytes)
        P = self._params(None, payload_words=int(payload_words), map_words=int(map_words))
        if restore and cover is None:
            cover = torch.empty((self.B, self.H, self.W), dtype=_pix_dtype(self.out_bytes), device=self.device)
        if payload is None:
            payload = torch.empty((self.B, int(payload_words)), dtype=torch.int64, device=self.device)
        lib = _lib.load()
        _lib.check(lib.codec_extract(C.byref(P), stego.data_ptr(), maps.data_ptr(), meta.data_ptr(),
                                     cover.data_ptr() if restore else None, payload.data_ptr(), _stream()),
                   "codec_extract")
        return payload, cover

    def decode_ref_compat_bits(self, stego, maps, meta, *, map_words: int):
        """decode_message bit streams: (bits uint8 [B, cap], counts int32 [B]) on device."""
        torch = _torch()
        P = self._params(None, map_words=int(map_words))
        cap = int(map_words) * 64
        bits = torch.zeros((self.B, cap), dtype=torch.uint8, device=self.device)
        counts = torch.zeros((self.B,), dtype=torch.int32, device=self.device)
        lib = _lib.load()
        _lib.check(lib.codec_refdecode(C.byref(P), stego.data_ptr(), maps.data_ptr(), meta.data_ptr(),
                                       bits.data_ptr(), cap, counts.data_ptr(), _stream()), "codec_refdecode")
        return bits, counts

    def expand_maps(self, maps, meta, *, map_words: int, smax: int = 16):
        torch = _torch()
        P = self._params(None, map_words=int(map_words))
        dense = torch.empty((self.B, smax, self.H, self.W), dtype=torch.uint8, device=self.device)
        _lib.check(_lib.load().codec_expand_maps(C.byref(P), maps.data_ptr(), meta.data_ptr(), dense.data_ptr(),
                                                 int(smax), _stream()), "codec_expand_maps")
        return dense


# ------------------------------------------------------------------ functional API
_CODECS = {}


def _codec_for(shape, dtype, **kw) -> Codec:
    torch = _torch()
    key = (tuple(shape), str(dtype), tuple(sorted(kw.items())), torch.cuda.current_device())
    c = _CODECS.get(key)
    if c is None:
        c = Codec(*shape, dtype=dtype, **kw)
        _CODECS[key] = c
    return c


def _as_batch(covers):
    torch = _torch()
    if isinstance(covers, np.ndarray):
        if covers.dtype not in (np.uint8, np.uint16):
            raise ValueError("A imagem deve ser uint8 ou uint16.")
        covers = torch.from_numpy(np.ascontiguousarray(covers)).cuda()
    if covers.dim() == 2:
        covers = covers.unsqueeze(0)
    if covers.dim() != 3:
        raise ValueError("A imagem deve ser 2D (grayscale).")   # codec.py:34
    return covers.contiguous()


def encode(covers, payloads: Sequence, *, method: str = "lsb", beta: float = 0.4, block: int = 16,
           align: bool = False, mode: str = "hybrid", nbits: Optional[int] = None, T=2, tmax: int = 16,
           maxval: Optional[int] = None, scheme: int = 1):
    """Embed one payload per slice.

    method="lsb" (default): the reference's bit-plane scheme, bit-exact with src/codec.py;
    defaults are main()'s (codec.py:868 beta=0.4, codec.py:875 search_block_size=16).
    Returns an Encoded.
    method="pee": MED-predictor prediction-error expansion (the north star's algorithm; the
    reference has none): T = expansion threshold or "auto" (capacity control,
    smallest T <= tmax per slice), maxval = largest legal pixel value (4095 for 12-bit data),
    scheme = 1 (the (odd, odd) lattice) or 2 (four sublattice passes, integer T).
    Returns a pee.PeeEncoded; beta/block/align/mode/nbits do not apply.
    decode() takes either result."""
    if method == "pee":
        from . import pee
        return pee.encode(covers, payloads, T=T, tmax=tmax, maxval=maxval, scheme=scheme)
    if method != "lsb":
        raise ValueError("method must be 'lsb' or 'pee'")
    _require_gpu()
    covers = _as_batch(covers)
    if isinstance(payloads, (str, bytes, bytearray)):
        payloads = [payloads]
    codec = _codec_for(tuple(covers.shape), str(covers.dtype), beta=beta, block=block, align=align,
                       mode=mode, nbits=nbits)
    return codec.encode(covers, payloads)


def decode(enc, *, restore: bool = True):
    """True extraction.  Returns (payload_bit_lists, cover) where payload_bit_lists[b] is a
    numpy 0/1 vector of the embedded bits in message order and cover the restored [B,H,W]
    (LSB: positional recovery; MED-PEE: the exact inverse)."""
    from . import pee
    if isinstance(enc, pee.PeeEncoded):
        return pee.decode(enc, restore=restore)
    _require_gpu()
    c = _codec_for(tuple(enc.stego.shape), _in_dtype_name(enc), **_codec_kw(enc))
    words, cover = c.decode(enc.stego, enc.maps, enc.meta, payload_words=enc.payloads.payload_words,
                            map_words=enc.payloads.map_words, restore=restore)
    recs = meta_records(enc.meta)
    host = words.cpu().numpy()
    bits = [framing.unpack_bits(host[b], recs[b].total_used) for b in range(len(recs))]
    return bits, cover


def decode_ref_compat(enc: Encoded) -> List[str]:
    """The reference's decode_message() output string per slice (codec.py:752-787),
    bit-exact including its lossy behaviour."""
    _require_gpu()
    c = _codec_for(tuple(enc.stego.shape), _in_dtype_name(enc), **_codec_kw(enc))
    bits, counts = c.decode_ref_compat_bits(enc.stego, enc.maps, enc.meta, map_words=enc.payloads.map_words)
    hb = bits.cpu().numpy()
    hc = counts.cpu().numpy()
    return [framing.bits_to_bytes_msb(hb[b, : hc[b]]).decode("utf-8", errors="replace") for b in range(hb.shape[0])]


def _in_dtype_name(enc: Encoded) -> str:
    # decode runs on the stego dtype; stego and cover share it in the default config
    return str(enc.stego.dtype)


def _codec_kw(enc: Encoded) -> dict:
    cfg = enc.config
    return dict(beta=cfg["beta"], block=cfg["block"], align=cfg["align"], mode=cfg["mode"], nbits=cfg["nbits"])
