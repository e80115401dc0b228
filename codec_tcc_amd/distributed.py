"""Multi-GPU sharding of a slice batch.

Slices are independent (s, offset, plan and maps are per slice: codec.py:561-599,
412-487; the MED-PEE side information T, L, end and the location map are per slice too),
so rank r simply encodes/decodes its own contiguous share with no data-path collective
("weak" scaling).  The one exchange the north star asks for -- every rank holding every
slice's location map -- is an `all_gather_into_tensor` of fixed-size records:

* LSB path (`RecordExchange`): codec_slice_meta + packed maps, ~1.6 KB per slice, one
  collective; never the dense s*H*W bitmaps (335 MB for 2048 x 512^2).
* MED-PEE path (`PeeRecordExchange`): one collective of records = the 64-byte
  codec_pee_meta of every slice + its location map, sparse (candidate indices of the set
  bits) or dense up to `end`, whichever the job-wide width holds (codec_pee_pack_records);
  the width is agreed once and then carried from step to step without a host sync (the
  device checks every gather against the width its metas needed; see the class).

Uneven shards (e.g. 2049 slices over 8 ranks) are padded to ceil(N / world) rows per
rank, the collective stays one equal-sized all-gather, and the padding rows are dropped
on the way out.  Backend "nccl" is RCCL on ROCm (xGMI between the 8 MI355X); "gloo" is
used by the CPU tests.  Everything here is shape/bookkeeping code: the kernels stay in
codec.py / pee.py.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

from . import _lib


def shard_range(n_items: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split [lo, hi) of n_items over `world` ranks (sizes differ by <= 1)."""
    base, extra = divmod(int(n_items), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_rows(n_items: int, world: int) -> int:
    """Rows every rank contributes to a gather: the largest shard (ceil(n / world))."""
    return max(1, -(-int(n_items) // int(world)))


def valid_rows(n_items: int, world: int) -> List[int]:
    """Indices of the real (non-padding) rows of a padded gather, in global slice order."""
    rows = shard_rows(n_items, world)
    out = []
    for r in range(world):
        lo, hi = shard_range(n_items, world, r)
        out.extend(r * rows + i for i in range(hi - lo))
    return out


def record_words(map_words: int) -> int:
    """int64 words per slice record: meta (rounded up to 8 B) + packed location map."""
    return (_lib.META_BYTES + 7) // 8 + int(map_words)


def pack_records(meta, maps, out=None):
    """[B, META_BYTES] uint8 + [B, map_words] int64 -> [B, record_words] int64.
    `out` may be wider than the maps (a job-wide map width): the extra words are zero."""
    import torch
    B = meta.shape[0]
    mw = maps.shape[1]
    hdr = (_lib.META_BYTES + 7) // 8
    if out is None:
        out = torch.zeros((B, record_words(mw)), dtype=torch.int64, device=meta.device)
    out[:B, :hdr].view(torch.uint8)[:, : _lib.META_BYTES].copy_(meta)
    out[:B, hdr: hdr + mw].copy_(maps)
    if out.shape[1] > hdr + mw:
        out[:B, hdr + mw:].zero_()
    return out


def unpack_records(records, map_words: int):
    """Inverse of pack_records: (meta uint8 [N, META_BYTES], maps int64 [N, map_words])."""
    hdr = (_lib.META_BYTES + 7) // 8
    import torch
    meta = records[:, :hdr].contiguous().view(torch.uint8)[:, : _lib.META_BYTES]
    maps = records[:, hdr: hdr + int(map_words)]
    return meta.contiguous(), maps.contiguous()


def _is_gloo(group) -> bool:
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


def agree_max(value: int, group=None, device=None) -> int:
    """The maximum of an integer over all ranks (one tiny all_reduce; host value out)."""
    import torch
    import torch.distributed as dist
    dev = "cpu" if (device is None or _is_gloo(group)) else device
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def gather_records(local_records, group=None, out=None, rows: Optional[int] = None):
    """all_gather_into_tensor of every rank's records -> [world * rows, W] (rank-major).

    `rows` (default: this rank's row count) is the per-rank row count of the collective;
    a shorter local shard is zero-padded to it, so uneven shards still make one
    equal-sized collective (drop the padding with `valid_rows`)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n, width = local_records.shape
    rows = n if rows is None else int(rows)
    if n > rows:
        raise ValueError(f"local shard of {n} rows exceeds the per-rank row count {rows}")
    src = local_records
    if n < rows or not src.is_contiguous():
        src = torch.zeros((rows, width), dtype=local_records.dtype, device=local_records.device)
        src[:n].copy_(local_records)
    if out is None:
        out = torch.empty((world * rows, width), dtype=local_records.dtype, device=local_records.device)
    if _is_gloo(group):
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, src, group=group)
        if parts[0].data_ptr() != out.data_ptr():   # chunk() views: already in place
            torch.cat(parts, 0, out=out)
    else:
        dist.all_gather_into_tensor(out, src, group=group)
    return out


class _SideStream:
    """Runs an exchange on a side stream that waits only for the point after encode, so
    decode's kernels keep the launch stream busy meanwhile (no-op on CPU tensors)."""

    def __init__(self, device):
        import torch
        dev = torch.device(device)
        self.device = dev
        self.stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self.event = torch.cuda.Event() if self.stream is not None else None
        self._marked = False

    def mark(self):
        import torch
        if self.stream is not None:
            self.event.record(torch.cuda.current_stream(self.device))
            self._marked = True

    def enter(self):
        import contextlib

        import torch
        if self.stream is None:
            return contextlib.nullcontext()
        if self._marked:
            self.stream.wait_event(self.event)
            self._marked = False
        else:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
        return torch.cuda.stream(self.stream)

    def join(self):
        import torch
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)


class RecordExchange:
    """The LSB record all-gather of one batch, overlapped with that batch's decode.

    The records depend only on what encode wrote (meta + packed maps), so they are packed
    and gathered on a side stream while decode's kernels run on the launch stream:
    ``mark()`` right after encode is queued (records an event), then decode, then
    ``start(meta, maps)`` (the side stream waits for the event only, so a host-blocking
    backend such as gloo does not hold back decode's launches either), and ``join()`` (the
    current stream waits for the gather, so the next encode cannot overwrite meta/maps under
    the pack).  On RCCL the collective runs on its own stream ordered after the side stream.
    CPU tensors (gloo tests) run synchronously.

    ``n_total`` (default batch * world) is the job's slice count; with uneven shards every
    rank pads to ceil(n_total / world) rows.  The map width is agreed as the job-wide
    maximum at construction (one all_reduce), since payload lengths -- and so the map
    words -- may differ per rank."""

    def __init__(self, batch: int, map_words: int, world: int, device, group=None, n_total: Optional[int] = None):
        import torch
        self.group = group
        self.world = int(world)
        self.n_total = int(n_total) if n_total is not None else int(batch) * self.world
        self.rows = shard_rows(self.n_total, self.world)
        if batch > self.rows:
            raise ValueError("batch exceeds the per-rank row count of n_total")
        self.batch = int(batch)
        self.map_words = agree_max(map_words, group, device) if self.world > 1 else int(map_words)
        words = record_words(self.map_words)
        self.record = torch.zeros((self.rows, words), dtype=torch.int64, device=device)
        self.padded = torch.empty((self.world * self.rows, words), dtype=torch.int64, device=device)
        self.even = self.rows * self.world == self.n_total
        self.index = None if self.even else torch.tensor(valid_rows(self.n_total, self.world), device=device)
        self._side = _SideStream(device)

    @property
    def gathered(self):
        """[n_total, words] records in global slice order (a view when shards are even)."""
        return self.padded if self.even else self.padded.index_select(0, self.index)

    def own_rows(self, rank: int):
        """This rank's rows of the gathered (padded) buffer."""
        return self.padded[rank * self.rows: rank * self.rows + self.batch]

    def mark(self):
        """Record the point after encode on the current stream (no-op on CPU)."""
        self._side.mark()

    def start(self, meta, maps):
        with self._side.enter():
            pack_records(meta, maps, out=self.record)
            gather_records(self.record, self.group, out=self.padded, rows=self.rows)

    def join(self):
        self._side.join()
        return self.gathered


PEE_META_WORDS = (_lib.PEE_META_BYTES + 7) // 8
PEE_END_FIELD = 3          # int32 index of codec_pee_meta.end
PEE_LMCOUNT_FIELD = 9      # int32 index of codec_pee_meta.lm_count
PEE_FLAGS_FIELD = 12       # int32 index of codec_pee_meta.flags
RECORD_RECOUNTED = 2       # CODEC_PEE_RECORD_RECOUNTED
assert PEE_META_WORDS == _lib.PEE_RECORD_HDR_WORDS


def map_prefix(meta, lm, lmw: int, out=None):
    """The first `lmw` location-map words of every slice with every bit past its own `end`
    cleared (the embed leaves the words past ceil((end + 1) / 64) unwritten) -- the map as a
    gathered record carries it."""
    import torch
    ends = meta.contiguous().view(torch.int32)[:, PEE_END_FIELD].to(torch.int64)
    nbits = torch.clamp(ends[:, None] + 1 - 64 * torch.arange(lmw, device=lm.device, dtype=torch.int64)[None, :], 0, 64)
    keep = torch.where(nbits >= 64, torch.full_like(nbits, -1),
                       (torch.ones_like(nbits) << nbits) - 1)            # low nbits of each word
    if out is None:
        out = torch.empty((lm.shape[0], lmw), dtype=torch.int64, device=lm.device)
    return torch.bitwise_and(lm[:, :lmw], keep, out=out)


def record_width_needed(meta, cap: Optional[int] = None):
    """Device int64 scalar: the record width (map words) that carries every one of these
    slices' maps exactly -- max over slices of min(ceil(lm_count / 2), ceil((end + 1) / 64)),
    at least 1, at most `cap` (codec_pee_pack_records' rule; no host read)."""
    import torch
    m = meta.contiguous().view(torch.int32)
    end = m[:, PEE_END_FIELD].to(torch.int64)
    cnt = m[:, PEE_LMCOUNT_FIELD].to(torch.int64)
    need = torch.minimum(torch.div(cnt + 1, 2, rounding_mode="floor"),
                         torch.div(end + 64, 64, rounding_mode="floor"))
    w = need.max() if need.numel() else torch.zeros((), dtype=torch.int64, device=meta.device)
    w = torch.clamp(w, min=1)
    return torch.clamp(w, max=int(cap)) if cap is not None else w


def dense_words_needed(meta):
    """Device int64 scalar: ceil((max end + 1) / 64), the dense prefix every map fits in."""
    import torch
    e = meta.contiguous().view(torch.int32)[:, PEE_END_FIELD].to(torch.int64)
    return torch.clamp(torch.div(e.max() + 64, 64, rounding_mode="floor"), min=1) if e.numel() else \
        torch.ones((), dtype=torch.int64, device=meta.device)


def pack_pee_records(meta, lm, width: int, out=None):
    """[B, 64] uint8 metas + [B, lm_words] int64 maps -> [B, 8 + width] int64 records
    (codec_pee_pack_records: the meta, then the map sparse -- ascending candidate indices of
    its set bits -- when lm_count <= 2 * width, else dense, bits past `end` cleared).  CUDA
    tensors run the HIP kernel; CPU tensors (the gloo tests' synthetic records) a row loop
    of the same rule."""
    import torch
    if meta.dtype != torch.uint8 or meta.dim() != 2 or int(meta.shape[1]) != _lib.PEE_META_BYTES:
        raise ValueError(f"meta must be uint8 [B, {_lib.PEE_META_BYTES}], got {meta.dtype} {tuple(meta.shape)}")
    if lm.dtype != torch.int64 or lm.dim() != 2 or int(lm.shape[0]) != int(meta.shape[0]):
        raise ValueError(f"lm must be int64 [B, lm_words] with B = {int(meta.shape[0])}, got {lm.dtype} {tuple(lm.shape)}")
    meta, lm = meta.contiguous(), lm.contiguous()   # a sliced view must not reach the kernel
    B, lmw = int(meta.shape[0]), int(lm.shape[1])
    if out is None:
        out = torch.empty((B, PEE_META_WORDS + int(width)), dtype=torch.int64, device=meta.device)
    if meta.is_cuda:
        from .codec import _stream
        _lib.check(_lib.load().codec_pee_pack_records(B, lmw, meta.data_ptr(), lm.data_ptr(), int(width),
                                                      out.data_ptr(), _stream()), "codec_pee_pack_records")
        return out
    import numpy as np
    out.zero_()
    out[:, :PEE_META_WORDS].view(torch.uint8)[:, : _lib.PEE_META_BYTES].copy_(meta)
    m = meta.contiguous().view(torch.int32)
    pref = map_prefix(meta, lm, lmw).numpy().view(np.uint64)
    for b in range(B):
        cnt = int(m[b, PEE_LMCOUNT_FIELD])
        if 0 <= cnt <= 2 * width:
            bits = np.unpackbits(pref[b].view(np.uint8), bitorder="little")
            idx = np.flatnonzero(bits)[:cnt].astype(np.uint32)
            slots = np.zeros(2 * width, dtype=np.uint32)
            slots[: idx.size] = idx
            out[b, PEE_META_WORDS:] = torch.from_numpy(slots.view(np.int64))
            if idx.size < cnt:   # fewer bits than lm_count says: the kernel's recount rule
                hdr = out[b, :PEE_META_WORDS].view(torch.int32)
                hdr[PEE_LMCOUNT_FIELD] = int(idx.size)
                hdr[PEE_FLAGS_FIELD] |= RECORD_RECOUNTED
        else:
            n = min(width, lmw)
            out[b, PEE_META_WORDS: PEE_META_WORDS + n] = torch.from_numpy(pref[b, :n].view(np.int64))
    return out


def unpack_pee_records(records, lm_cols: int, out=None):
    """[n, 8 + width] records -> (meta uint8 [n, 64], lm int64 [n, lm_cols]): every slice's
    map dense, zero past its `end` (codec_pee_unpack_records on CUDA tensors)."""
    import torch
    n, width = int(records.shape[0]), int(records.shape[1]) - PEE_META_WORDS
    meta = records[:, :PEE_META_WORDS].contiguous().view(torch.uint8)[:, : _lib.PEE_META_BYTES]
    if out is None:
        out = torch.empty((n, int(lm_cols)), dtype=torch.int64, device=records.device)
    if records.is_cuda:
        from .codec import _stream
        rec = records.contiguous()
        _lib.check(_lib.load().codec_pee_unpack_records(n, width, rec.data_ptr(), int(lm_cols), None,
                                                        out.data_ptr(), _stream()), "codec_pee_unpack_records")
        return meta, out
    import numpy as np
    out.zero_()
    m = meta.contiguous().view(torch.int32)
    for b in range(n):
        cnt = int(m[b, PEE_LMCOUNT_FIELD])
        pay = records[b, PEE_META_WORDS:].numpy()
        if 0 <= cnt <= 2 * width:
            idx = pay.view(np.uint32)[:cnt].astype(np.int64)
            idx = idx[idx < 64 * lm_cols]
            bits = np.zeros(64 * lm_cols, dtype=np.uint8)
            bits[idx] = 1
            out[b] = torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int64))
        else:
            dw = min(width, lm_cols, max(0, (int(m[b, PEE_END_FIELD]) + 64) // 64))
            out[b, :dw] = records[b, PEE_META_WORDS: PEE_META_WORDS + dw]
    return meta, out


class PeeRecordExchange:
    """The MED-PEE side information of every slice to every rank (north star: "an RCCL
    all-gather of per-slice location maps").

    One collective per step of fixed-width records (codec_pee_pack_records): every slice's
    64-byte codec_pee_meta (T, L, end, maxval, status, capacity, lm_count ...) followed by
    `width` words of its location map -- sparse (the candidate indices of its set bits) when
    lm_count <= 2 * width, else the dense prefix up to `end`.  Real maps are nearly empty
    (only overflow-prone candidates are set), so a 2048^2 ct12 slice's record is 72 bytes
    where the dense prefix was ~15.8 KB.

    The width that carries every map exactly is the job-wide max of
    min(ceil(lm_count / 2), ceil((end + 1) / 64)) -- a device value.  Reading it every step
    would block the host on the side stream, so it is carried over (no host sync in start()):
    * the first gather agrees it exactly: metas first, one host read, then the records;
    * every gather computes, on the device, the width its own metas needed, bumps a sticky
      device counter (``overflows()``) when it exceeded the width used, and copies the figure
      into pinned host memory behind an event; a later ``start`` adopts a larger width as
      soon as that event has completed (``Event.query``, never a wait);
    * ``join()`` is exact: one host read, a re-gather at the wider width if this step's
      maps did not fit (never cut-short rows by default), then the dense maps;
    * ``join_records()`` is the benchmark's opt-in: no host read, the raw gathered records,
      exact only if ``overflows()`` reads 0 afterwards.
    Uneven shards are padded as in RecordExchange."""

    def __init__(self, batch: int, world: int, device, group=None, n_total: Optional[int] = None,
                 width: Optional[int] = None):
        import torch
        self.group = group
        self.world = int(world)
        self.n_total = int(n_total) if n_total is not None else int(batch) * self.world
        self.rows = shard_rows(self.n_total, self.world)
        if batch > self.rows:
            raise ValueError("batch exceeds the per-rank row count of n_total")
        self.batch = int(batch)
        self.device = torch.device(device)
        self.even = self.rows * self.world == self.n_total
        self.index = None if self.even else torch.tensor(valid_rows(self.n_total, self.world), device=device)
        self.width = int(width) if width else 0
        self._rec_flat = None
        self._out_flat = None
        self._rec = self._out = None
        self._dense = None
        self._cuda = self.device.type == "cuda"
        self._need = torch.zeros(2, dtype=torch.int64, device=device)       # [record width, dense words]
        self._overflow = torch.zeros((), dtype=torch.int64, device=device)
        self._need_host = torch.zeros(2, dtype=torch.int64, pin_memory=self._cuda)
        self._need_ev = torch.cuda.Event() if self._cuda else None
        self._pending = False
        self._last = None
        self._side = _SideStream(device)

    # -- buffers: [rows, META_WORDS + width] records, [world * rows, ...] gathered
    def _buffers(self, width: int):
        import torch
        w = PEE_META_WORDS + width
        need = self.rows * w
        if self._rec_flat is None or self._rec_flat.numel() < need:
            self._rec_flat = torch.zeros(need, dtype=torch.int64, device=self.device)
            self._out_flat = torch.empty(self.world * need, dtype=torch.int64, device=self.device)
        self._rec = self._rec_flat[:need].view(self.rows, w)
        self._out = self._out_flat[: self.world * need].view(self.world * self.rows, w)
        return self._rec, self._out

    @property
    def lm_words(self) -> int:
        """Map words per gathered record (the carried width)."""
        return self.width

    @property
    def record_bytes(self) -> int:
        """Bytes per slice record of the last gather (meta + map payload)."""
        return (PEE_META_WORDS + self.width) * 8

    @property
    def gathered_bytes(self) -> int:
        """Bytes every rank receives per gather."""
        return 0 if self._out is None else int(self._out.numel()) * 8

    @property
    def meta_padded(self):
        return self._out[:, :PEE_META_WORDS]

    def mark(self):
        self._side.mark()

    def _adopt_width(self, cap: int):
        """Take a wider width from an earlier gather whose figure has landed on the host."""
        if self._pending and (self._need_ev is None or self._need_ev.query()):
            need = int(self._need_host[0])
            self._pending = False
            if need > self.width:
                self.width = min(need, cap)

    def _gather(self, meta, lm, width: int):
        """Pack the records (HIP kernel) and gather them (side stream)."""
        import torch
        B = meta.shape[0]
        rec, out = self._buffers(width)
        pack_pee_records(meta, lm, width, out=rec[:B])
        if B < self.rows:
            rec[B:].zero_()
        gather_records(rec, self.group, out=out, rows=self.rows)
        # the widths this gather needed, over the whole job (every rank computes the same)
        gm = out[:, :PEE_META_WORDS].contiguous().view(torch.uint8)
        if not self.even:
            gm = gm.index_select(0, self.index)
        self._need[0].copy_(record_width_needed(gm, int(lm.shape[1])))
        self._need[1].copy_(dense_words_needed(gm))
        self._overflow.add_((self._need[0] > width).to(torch.int64))
        self._need_host.copy_(self._need, non_blocking=self._cuda)
        if self._need_ev is not None:
            self._need_ev.record()
        self._pending = True

    def start(self, meta, lm):
        """meta: uint8 [B, PEE_META_BYTES]; lm: int64 [B, lm_words] (PeeCodec outputs).
        Queues the gather on the side stream; the host never waits on the device here except
        on the very first call (the exact initial width)."""
        import torch
        cap = int(lm.shape[1])
        self._adopt_width(cap)
        self._last = (meta, lm)
        with self._side.enter():
            if self.width <= 0:
                # first call: agree the width exactly (metas first, one host read)
                rec, _ = self._buffers(1)
                rec[: meta.shape[0], :PEE_META_WORDS].view(torch.uint8)[:, : _lib.PEE_META_BYTES].copy_(meta)
                if meta.shape[0] < self.rows:
                    rec[meta.shape[0]:].zero_()
                mout = gather_records(rec[:, :PEE_META_WORDS].contiguous(), self.group, rows=self.rows)
                self.width = int(record_width_needed(mout.view(torch.uint8), cap).item())
            self.width = min(self.width, cap)
            self._gather(meta, lm, self.width)

    def verify(self) -> bool:
        """One host read: did the last gather carry every map?  If not, re-gather it at the
        needed width (meta/lm of that step must still be intact) and keep that width.
        Returns True when the last gather had to be repeated."""
        if self._last is None:
            return False
        self._side.join()
        need = int(self._need[0].item())
        if need <= self.width:
            return False
        meta, lm = self._last
        self.width = min(need, int(lm.shape[1]))
        with self._side.enter():
            self._gather(meta, lm, self.width)
            self._overflow.sub_(1)   # repaired: this step's records are now complete
        return True

    def overflows(self) -> int:
        """Gathers (since construction) whose width was too narrow and not repaired by
        verify(): some of their maps were cut short (one host read)."""
        self._side.join()
        return int(self._overflow.item())

    def own_rows(self, rank: int):
        """This rank's rows of the gathered (padded) records."""
        a = rank * self.rows
        return self._out[a: a + self.batch]

    def join_records(self):
        """The gathered records [n_total, 8 + width] in global slice order, without any host
        read (benchmarks; check overflows() == 0 afterwards).  Decode a row with
        unpack_pee_records."""
        self._side.join()
        return self._out if self.even else self._out.index_select(0, self.index)

    def join(self):
        """(meta uint8 [n_total, PEE_META_BYTES], lm int64 [n_total, words]) in global slice
        order, exact: every slice's location map dense up to the job's largest `end` (words =
        ceil((max end + 1) / 64)), zero past its own end.  One host read (verify())."""
        import torch
        self.verify()
        self._side.join()
        cols = int(self._need[1].item())
        rec = self._out if self.even else self._out.index_select(0, self.index)
        if self._dense is None or self._dense.numel() < rec.shape[0] * cols:
            self._dense = torch.empty(rec.shape[0] * cols, dtype=torch.int64, device=self.device)
        meta, lm = unpack_pee_records(rec, cols, out=self._dense[: rec.shape[0] * cols].view(rec.shape[0], cols))
        return meta.contiguous(), lm
