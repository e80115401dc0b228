"""Drop-in functions with the reference's names, argument meaning and return types
(numpy in, numpy out), each running on the MI355X through the C ABI.

    from codec_tcc_amd import api as codec     # instead of `import codec` (src/codec.py)

| reference (src/codec.py)                     | here                                    |
|----------------------------------------------|-----------------------------------------|
| message_to_bits                 :239-240     | host (framing.message_to_bits)          |
| distribute_message_segments     :242-274     | host (framing.distribute_message_segments) |
| calculate_entropy               :489-502     | codec_plan (histogram + exact entropy)  |
| calculate_mutual_information    :504-559     | codec_plan (all_mi)                     |
| adaptive_modalities_decomposition :561-599   | codec_plan + codec_unpack_planes        |
| lsb_embed_multi_plane           :276-318     | codec_merge_planes + plan + embed + expand |
| lsb_embed_block_then_multiplane :412-487     | codec_merge_planes + plan + embed + expand |
| lsb_embed_block_adaptive        :320-410     | codec_block_variance + host sort + codec_lsb_runs |
| merge_modalities                :215-237     | codec_merge_planes                      |
| extract_local_planes            :789-793     | codec_unpack_planes                     |
| decode_message                  :752-787     | codec_refdecode_dense                   |
| (new) decode_positional                      | restore_dense + plan + extract: the exact payload |

Differences, all raising instead of silently diverging: planes handed to the embedders
must hold 0/1 values (what adaptive_modalities_decomposition produces); images must be
uint8/uint16 (codec.py:36-37 enforces the same for DICOM output); nbits <= 16; and
calculate_mutual_information supports bit planes of the image (the reference's only use,
codec.py:588).  The reference's progress print()s are not reproduced.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np

from . import _lib, framing
from .codec import Codec, _require_gpu, _stream, _torch, make_payloads, meta_records
from .framing import distribute_message_segments, message_to_bits  # noqa: F401  (re-export)

__all__ = [
    "message_to_bits", "distribute_message_segments", "calculate_entropy", "calculate_mutual_information",
    "adaptive_modalities_decomposition", "lsb_embed_multi_plane", "lsb_embed_block_then_multiplane",
    "lsb_embed_block_adaptive",
    "merge_modalities", "extract_local_planes", "decode_message", "decode_positional",
]


def _dev():
    return _torch().device("cuda", _torch().cuda.current_device())


def _to_dev(arr: np.ndarray):
    return _torch().from_numpy(np.ascontiguousarray(arr)).to(_dev())


def _as_pixels(a) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype == np.bool_:
        a = a.astype(np.uint8)
    if a.dtype not in (np.uint8, np.uint16):
        if a.dtype.kind in "iu" and a.size and a.min() >= 0 and a.max() <= 65535:
            a = a.astype(np.uint16)
        else:
            raise ValueError("A imagem deve ser uint8 ou uint16.")
    return a


def _params(B, H, W, in_bytes, out_bytes, **kw):
    P = _lib.Params(B=B, H=H, W=W, in_bytes=in_bytes, out_bytes=out_bytes, nbits=kw.get("nbits", 8 * in_bytes),
                    block=1, align=0, mode=0, fixed_s=0, fixed_offset=-1, all_mi=0, payload_words=1,
                    map_words=kw.get("map_words", 1), n_classes=1, reserved=0, beta=0.0)
    return P


def _planes_stack(planes: Sequence[np.ndarray], need01: bool):
    arrs = [np.asarray(p) for p in planes]
    if not arrs:
        raise ValueError("no planes")
    shape = arrs[0].shape
    if any(a.shape != shape for a in arrs):
        raise ValueError("all planes must share a shape")
    dt = arrs[0].dtype
    st = np.stack(arrs, axis=0)
    if need01 and st.size and (st.min() < 0 or st.max() > 1):
        raise ValueError("local planes must hold 0/1 values (as adaptive_modalities_decomposition returns)")
    if st.dtype not in (np.uint8, np.uint16):
        st = st.astype(np.uint16 if st.size and st.max() > 255 else np.uint8)
    return st, shape, dt


def _info(image: np.ndarray, *, all_mi: bool, beta: float = 0.8, nbits=None):
    img = _as_pixels(image)
    n = img.size
    if n == 0:
        raise ValueError("zero-size array")
    codec = Codec(1, 1, n, dtype=str(img.dtype), beta=beta, block=16, mode="multi", nbits=nbits,
                  all_mi=all_mi)
    meta = codec.plan(_to_dev(img.reshape(1, 1, n)), [np.zeros(0, np.uint8)])
    return meta_records(meta)[0], img


# ------------------------------------------------------------------ information theory
def calculate_entropy(data_array) -> float:
    """codec.py:489-502, bit-exact (device histogram, numpy-order float64 sum)."""
    _require_gpu()
    m, _ = _info(data_array, all_mi=False)
    return float(m.entropy)


def calculate_mutual_information(bit_plane, image_array) -> float:
    """codec.py:504-559 for X = a bit plane of Y (how codec.py:588 calls it)."""
    _require_gpu()
    x = np.asarray(bit_plane)
    y = _as_pixels(image_array)
    if x.size != y.size:
        raise ValueError("bit_plane and image_array must have the same size")
    if x.min() == x.max() or y.min() == y.max():          # codec.py:520-523
        return 0.0
    torch = _torch()
    yt = _to_dev(y.reshape(-1).astype(np.int32))
    xt = _to_dev(x.reshape(-1).astype(np.int32))
    plane = -1
    for i in range(8 * y.dtype.itemsize):
        if bool(torch.equal((yt >> i) & 1, xt)):
            plane = i
            break
    if plane < 0:
        raise NotImplementedError("calculate_mutual_information: bit_plane must be a bit plane of image_array")
    m, _ = _info(y, all_mi=True, nbits=8 * y.dtype.itemsize)
    return float(m.mi[plane])


def adaptive_modalities_decomposition(image_array, beta=0.8, nbits=None):
    """codec.py:561-599 -> (global_planes, local_planes), planes in the image dtype."""
    _require_gpu()
    img = np.asarray(image_array)
    if img.dtype not in (np.uint8, np.uint16):
        raise ValueError("A imagem deve ser uint8 ou uint16.")
    nb = img.dtype.itemsize * 8 if nbits is None else int(nbits)
    m, img = _info(img, all_mi=False, beta=beta, nbits=nb)
    s = m.s
    n = img.size
    torch = _torch()
    planes = torch.empty((1, nb, n), dtype=torch.uint16 if img.dtype == np.uint16 else torch.uint8, device=_dev())
    P = _params(1, 1, n, img.dtype.itemsize, img.dtype.itemsize)
    src = _to_dev(img.reshape(1, 1, n))
    _lib.check(_lib.load().codec_unpack_planes(C.byref(P), src.data_ptr(), 0, nb, planes.data_ptr(),
                                               img.dtype.itemsize, _stream()), "codec_unpack_planes")
    host = planes.cpu().numpy()[0]
    pl = [host[i].reshape(img.shape) for i in range(nb)]
    return pl[s:], pl[:s]


# ------------------------------------------------------------------ embedding
def _embed(local_planes, message_bits: str, *, mode: str, block: int, align: bool):
    _require_gpu()
    st, shape, dt = _planes_stack(local_planes, need01=True)
    if len(shape) != 2:
        raise ValueError("planes must be 2-D (H, W)")
    s = st.shape[0]
    if s > 16:
        raise ValueError("at most 16 local planes")
    h, w = shape
    if any(ch not in "01" for ch in message_bits):
        raise ValueError("message_bits must be a '0'/'1' string")
    torch = _torch()
    dev = _dev()
    # pack the planes into one uint16 image whose bit p is plane p (codec_merge_planes)
    planes_t = _to_dev(st.reshape(1, s, h * w))
    cover = torch.empty((1, h, w), dtype=torch.uint16, device=dev)
    P = _params(1, h, w, 2, 2)
    _lib.check(_lib.load().codec_merge_planes(C.byref(P), planes_t.data_ptr(), s, st.dtype.itemsize,
                                              cover.data_ptr(), _stream()), "codec_merge_planes")
    codec = Codec(1, h, w, dtype="uint16", beta=0.0, block=block, align=align, mode=mode, nbits=16, fixed_s=s)
    bits = np.frombuffer(message_bits.encode("ascii"), dtype=np.uint8) - ord("0")
    enc = codec.encode(cover, [bits])
    m = meta_records(enc.meta)[0]
    out = torch.empty((1, s, h * w), dtype=torch.uint16 if dt == np.uint16 else torch.uint8, device=dev)
    Pu = _params(1, h, w, 2, 2)
    _lib.check(_lib.load().codec_unpack_planes(C.byref(Pu), enc.stego.data_ptr(), 0, s, out.data_ptr(),
                                               out.element_size(), _stream()), "codec_unpack_planes")
    dense = codec.expand_maps(enc.maps, enc.meta, map_words=enc.payloads.map_words, smax=s)
    host_planes = out.cpu().numpy()[0]
    host_maps = dense.cpu().numpy()[0]
    stego_planes = [host_planes[p].reshape(h, w).astype(dt, copy=False) for p in range(s)]
    bitmaps = [host_maps[p] for p in range(s)]
    return (stego_planes, bitmaps, int(m.total_used), [int(m.sizes[p]) for p in range(s)],
            [int(m.perm[j]) for j in range(s)])


def lsb_embed_block_then_multiplane(local_planes, message_bits, search_block_size=8, align_across_planes: bool = False):
    """codec.py:412-487 -> (stego_planes, bitmaps, total_used, segments_lengths, segment_indices)."""
    return _embed(local_planes, message_bits, mode="hybrid", block=int(search_block_size),
                  align=bool(align_across_planes))


def lsb_embed_multi_plane(local_planes, message_bits):
    """codec.py:276-318 -> (stego_planes, bitmaps, total_used, segments_lengths, segment_indices)."""
    return _embed(local_planes, message_bits, mode="multi", block=16, align=False)


def lsb_embed_block_adaptive(local_planes, message_bits, block_size=8):
    """codec.py:320-410 -> (stego_planes, bitmaps, total_used, segments_lengths, segment_indices).

    Every block's float(np.var(block)) comes from the device (codec_block_variance,
    numpy-exact); each plane's blocks are ordered by a stable descending sort of those
    scores on the host (Python's `list.sort(reverse=True)` keeps equal scores in raster
    order, as numpy's stable argsort of the negated scores does); the segment's bits are
    walked over the blocks in that order and the writes go back to the device as runs
    (codec_lsb_runs).  The reference's ravel-copy quirk is reproduced: `ravel()` of a block
    view is a view only when the block is C-contiguous (one row high, or the full image
    width), so only those blocks are written (codec.py:383-384, 397-398), while the bits of
    every visited block are consumed (:402) and counted in segments_lengths (:406)."""
    _require_gpu()
    st, shape, dt = _planes_stack(local_planes, need01=True)
    if len(shape) != 2:
        raise ValueError("planes must be 2-D (H, W)")
    if any(ch not in "01" for ch in message_bits):
        raise ValueError("message_bits must be a '0'/'1' string")
    bs = int(block_size)
    if bs < 1:
        raise ValueError("block_size must be >= 1")     # range(0, h, 0) raises in the reference
    s = st.shape[0]
    h, w = shape
    n = h * w
    segments, _sizes, perm = framing.distribute_message_segments(list(local_planes), message_bits)
    torch = _torch()
    dev = _dev()
    nb = st.dtype.itemsize
    planes_t = _to_dev(st.reshape(s, n))
    nby, nbx = -(-h // bs), -(-w // bs)
    scores = torch.empty((s, nby * nbx), dtype=torch.float64, device=dev)
    lib = _lib.load()
    _lib.check(lib.codec_block_variance(s, h, w, nb, bs, planes_t.data_ptr(), scores.data_ptr(), _stream()),
               "codec_block_variance")
    sc = scores.cpu().numpy()
    by, bx = np.divmod(np.arange(nby * nbx, dtype=np.int64), nbx)
    bh = np.minimum(bs, h - by * bs)
    bw = np.minimum(bs, w - bx * bs)
    cap = bh * bw
    contiguous = (bh == 1) | (bw == w)
    first = by * bs * w + bx * bs
    lens = [0] * s
    used = 0
    runs = []
    seg_bits = np.zeros((s, max(1, max((min(len(g), n) for g in segments), default=0))), dtype=np.uint8)
    for seg, dest in zip(segments, perm):
        nseg = min(len(seg), n)                                       # codec.py:365
        if nseg:
            seg_bits[dest, :nseg] = np.frombuffer(seg[:nseg].encode("ascii"), dtype=np.uint8) - ord("0")
        order = np.argsort(-sc[dest], kind="stable")                  # codec.py:361
        c = cap[order]
        before = np.cumsum(c) - c                                     # bits consumed before each block
        visit = before < nseg                                         # codec.py:373-374
        k = np.minimum(nseg - before[visit], c[visit])
        cur = int(k.sum())
        lens[dest] = cur
        used += cur
        o = order[visit]
        wr = contiguous[o] & (k > 0)
        if wr.any():
            runs.append(np.stack([np.full(int(wr.sum()), dest, np.int64), first[o][wr], k[wr], before[visit][wr]], 1))
    out = planes_t
    bitmaps_t = torch.zeros((s, n), dtype=torch.uint8, device=dev)
    if runs:
        rr = np.ascontiguousarray(np.concatenate(runs, 0).astype(np.int64))
        runs_t = _to_dev(rr)
        bits_t = _to_dev(seg_bits)
        _lib.check(lib.codec_lsb_runs(s, n, nb, out.data_ptr(), bitmaps_t.data_ptr(), bits_t.data_ptr(),
                                      seg_bits.shape[1], runs_t.data_ptr(), rr.shape[0], _stream()), "codec_lsb_runs")
    host_planes = out.cpu().numpy()
    host_maps = bitmaps_t.cpu().numpy()
    stego_planes = [host_planes[p].reshape(h, w).astype(dt, copy=False) for p in range(s)]
    bitmaps = [host_maps[p].reshape(h, w) for p in range(s)]
    return stego_planes, bitmaps, used, lens, list(perm)


def merge_modalities(global_planes, local_planes) -> np.ndarray:
    """codec.py:215-237."""
    _require_gpu()
    planes = list(local_planes) + list(global_planes)
    total = len(planes)
    out_dt = np.uint16 if total > 8 else np.uint8
    arrs = [np.asarray(p) for p in planes]
    shape = arrs[0].shape
    norm = [a if a.dtype in (np.uint8, np.uint16) else a.astype(out_dt) for a in arrs]   # `.astype(dtype)`, :230/:234
    wide = any(a.dtype == np.uint16 for a in norm)
    st = np.stack([a.astype(np.uint16 if wide else np.uint8, copy=False) for a in norm], axis=0)
    n = int(np.prod(shape)) if shape else 1
    torch = _torch()
    out = torch.empty((1, n), dtype=torch.uint16 if out_dt == np.uint16 else torch.uint8, device=_dev())
    P = _params(1, 1, n, 1, 2 if out_dt == np.uint16 else 1)
    planes_t = _to_dev(st.reshape(1, total, n))
    _lib.check(_lib.load().codec_merge_planes(C.byref(P), planes_t.data_ptr(), total, st.dtype.itemsize,
                                              out.data_ptr(), _stream()), "codec_merge_planes")
    return out.cpu().numpy()[0].reshape(shape)


# ------------------------------------------------------------------ extraction
def extract_local_planes(stego_array, s):
    """codec.py:789-793."""
    _require_gpu()
    img = np.asarray(stego_array)
    if img.dtype not in (np.uint8, np.uint16):
        raise ValueError("A imagem deve ser uint8 ou uint16.")
    s = int(s)
    if s < 1:
        return []
    n = img.size
    torch = _torch()
    out = torch.empty((1, s, n), dtype=torch.uint16 if img.dtype == np.uint16 else torch.uint8, device=_dev())
    P = _params(1, 1, n, img.dtype.itemsize, img.dtype.itemsize)
    src_t = _to_dev(img.reshape(1, 1, n))
    _lib.check(_lib.load().codec_unpack_planes(C.byref(P), src_t.data_ptr(), 0, s, out.data_ptr(),
                                               img.dtype.itemsize, _stream()), "codec_unpack_planes")
    host = out.cpu().numpy()[0]
    return [host[i].reshape(img.shape) for i in range(s)]


def _meta_from_header(s: int, perm: Sequence[int], sizes: Sequence[int]):
    m = _lib.SliceMeta()
    m.s = s
    visited = set(int(p) for p in perm)
    for j in range(16):
        m.perm[j] = int(perm[j]) if j < len(perm) else -1
    for p in range(16):
        m.sizes[p] = int(sizes[p]) if (p < s and p in visited) else 0
    return m


def decode_message(stego_planes, bitmaps, metadata) -> str:
    """codec.py:752-787, including its lossy extraction."""
    _require_gpu()
    s = int(metadata["s"])
    if s < 1:
        return ""
    if s > 16:
        raise ValueError("at most 16 local planes")
    planes = [np.asarray(stego_planes[p]).reshape(-1) for p in range(s)]
    maps = [np.asarray(bitmaps[p]).reshape(-1) for p in range(s)]
    n = planes[0].size
    if any(p.size != n for p in planes) or any(b.size != n for b in maps):
        raise ValueError("planes and bitmaps must all have H*W elements")
    st = np.stack([(p & 1).astype(np.uint8) for p in planes], 0)
    dense = np.stack([(b != 0).astype(np.uint8) for b in maps], 0)
    m = _meta_from_header(s, metadata["segments_indices"], metadata["segments_lengths"])
    torch = _torch()
    meta = torch.frombuffer(bytearray(bytes(m)), dtype=torch.uint8).to(_dev()).view(1, -1)
    cap = 64 + sum(min(int(m.sizes[p]), n) if m.sizes[p] >= 0 else n for p in range(s))
    bits = torch.zeros((1, cap), dtype=torch.uint8, device=_dev())
    counts = torch.zeros((17,), dtype=torch.int32, device=_dev())
    P = _params(1, 1, n, 1, 1)
    # keep every device buffer referenced until the launch is enqueued: a temporary freed
    # mid-call returns its block to the caching allocator, which may hand it to the next
    # upload on the same stream before the kernel has read it
    src_t = _to_dev(st.reshape(1, s, n))
    dense_t = _to_dev(dense.reshape(1, s, n))
    _lib.check(_lib.load().codec_refdecode_dense(C.byref(P), src_t.data_ptr(), 1, dense_t.data_ptr(), s,
                                                 meta.data_ptr(), bits.data_ptr(), cap, counts.data_ptr(),
                                                 _stream()), "codec_refdecode_dense")
    k = int(counts[0].item())
    if k > cap:
        raise RuntimeError("decode_message: output capacity exceeded")
    return framing.bits_to_bytes_msb(bits.cpu().numpy()[0, :k]).decode("utf-8", errors="replace")


def decode_positional(stego_array, bitmaps, metadata, search_block_size: int = 16,
                      align_across_planes: bool = False, start_offset: Optional[int] = None):
    """Exact recovery from the reference's outputs.

    The dense bitmaps mark flipped LSBs only, so the cover is `stego ^ bitmaps`; the start
    offset is re-derived on the restored plane 0 exactly as the embedder derived it
    (codec.py:431-453) and the windows are read back in segment_indices order -- unless
    start_offset is given (a version-2 container stores the real one), which is then used
    as is.  Returns (message_bits as a '0'/'1' string, restored cover)."""
    _require_gpu()
    img = np.asarray(stego_array)
    if img.dtype not in (np.uint8, np.uint16) or img.ndim != 2:
        raise ValueError("stego must be a 2-D uint8/uint16 image")
    s = int(metadata["s"])
    perm = [int(x) for x in metadata["segments_indices"]]
    sizes = [int(x) for x in metadata["segments_lengths"]]
    h, w = img.shape
    n = h * w
    torch = _torch()
    dev = _dev()
    stego = _to_dev(img.reshape(1, h, w))
    dense = _to_dev(np.stack([(np.asarray(bitmaps[p]).reshape(-1) != 0).astype(np.uint8) for p in range(s)], 0)
                    .reshape(1, s, n))
    hb = img.dtype.itemsize
    cover = torch.empty((1, h, w), dtype=stego.dtype, device=dev)
    mrec = _lib.SliceMeta()
    mrec.s = s
    meta_in = torch.frombuffer(bytearray(bytes(mrec)), dtype=torch.uint8).to(dev).view(1, -1)
    P = _params(1, h, w, hb, hb)
    _lib.check(_lib.load().codec_restore_dense(C.byref(P), stego.data_ptr(), dense.data_ptr(), s, meta_in.data_ptr(),
                                               cover.data_ptr(), _stream()), "codec_restore_dense")
    total = sum(sizes)
    codec = Codec(1, h, w, dtype=str(img.dtype), beta=0.0, block=int(search_block_size),
                  align=bool(align_across_planes), mode="hybrid", fixed_s=s,
                  fixed_offset=-1 if start_offset is None else int(start_offset))
    pl = make_payloads([np.zeros(max(total, 0), np.uint8)], dev)
    meta = codec.plan(cover, pl)
    m = meta_records(meta)[0]
    if [m.perm[j] for j in range(s)] != perm:
        raise ValueError("segments_indices do not match the reference plan for s")
    payload, _ = codec.decode(stego, torch.zeros((1, pl.map_words), dtype=torch.int64, device=dev), meta,
                              payload_words=pl.payload_words, map_words=pl.map_words, restore=False)
    bits = framing.unpack_bits(payload.cpu().numpy()[0], m.total_used)
    return framing.bits_to_str(bits), cover.cpu().numpy()[0]
