"""Multi-GPU sharding of a slice batch.

Slices are independent (s, offset, plan and maps are per slice: codec.py:561-599,
412-487), so rank r simply encodes/decodes its own contiguous share with no data-path
collective ("weak" scaling).  The one exchange the north star asks for -- every rank
holding every slice's location map -- is ONE `all_gather_into_tensor` of fixed-size
records (codec_slice_meta + packed maps), latency-bound at ~1.6 KB per slice; never the
dense s*H*W bitmaps (335 MB for 2048 x 512^2).

Backend "nccl" is RCCL on ROCm (xGMI between the 8 MI355X); "gloo" is used by the CPU
tests.  Everything here is shape/bookkeeping code: the kernels stay in codec.py.
"""
from __future__ import annotations

from typing import Tuple

from . import _lib


def shard_range(n_items: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split [lo, hi) of n_items over `world` ranks (sizes differ by <= 1)."""
    base, extra = divmod(int(n_items), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def record_words(map_words: int) -> int:
    """int64 words per slice record: meta (rounded up to 8 B) + packed location map."""
    return (_lib.META_BYTES + 7) // 8 + int(map_words)


def pack_records(meta, maps, out=None):
    """[B, META_BYTES] uint8 + [B, map_words] int64 -> [B, record_words] int64."""
    import torch
    B = meta.shape[0]
    mw = maps.shape[1]
    words = record_words(mw)
    if out is None:
        out = torch.zeros((B, words), dtype=torch.int64, device=meta.device)
    hdr = (_lib.META_BYTES + 7) // 8
    out[:, :hdr].view(torch.uint8)[:, : _lib.META_BYTES].copy_(meta)
    out[:, hdr:].copy_(maps)
    return out


def unpack_records(records, map_words: int):
    """Inverse of pack_records: (meta uint8 [N, META_BYTES], maps int64 [N, map_words])."""
    hdr = (_lib.META_BYTES + 7) // 8
    import torch
    meta = records[:, :hdr].contiguous().view(torch.uint8)[:, : _lib.META_BYTES]
    maps = records[:, hdr: hdr + int(map_words)]
    return meta.contiguous(), maps.contiguous()


def gather_records(local_records, group=None, out=None):
    """all_gather_into_tensor of every rank's [B, W] records -> [world*B, W] (rank-major)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((world * local_records.shape[0], local_records.shape[1]), dtype=local_records.dtype,
                          device=local_records.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, local_records.contiguous(), group=group)
        if parts[0].data_ptr() != out.data_ptr():   # chunk() views: already in place
            torch.cat(parts, 0, out=out)
    else:
        dist.all_gather_into_tensor(out, local_records.contiguous(), group=group)
    return out


class RecordExchange:
    """The record all-gather of one batch, overlapped with that batch's decode.

    The records depend only on what encode wrote (meta + packed maps), so they are packed
    and gathered on a side stream while decode's kernels run on the launch stream:
    ``mark()`` right after encode is queued (records an event), then decode, then
    ``start(meta, maps)`` (the side stream waits for the event only, so a host-blocking
    backend such as gloo does not hold back decode's launches either), and ``join()`` (the
    current stream waits for the gather, so the next encode cannot overwrite meta/maps under
    the pack).  On RCCL the collective runs on its own stream ordered after the side stream.
    CPU tensors (gloo tests) run synchronously."""

    def __init__(self, batch: int, map_words: int, world: int, device, group=None):
        import torch
        self.group = group
        words = record_words(map_words)
        self.record = torch.zeros((batch, words), dtype=torch.int64, device=device)
        self.gathered = torch.empty((world * batch, words), dtype=torch.int64, device=device)
        dev = torch.device(device)
        self.stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self.event = torch.cuda.Event() if self.stream is not None else None
        self._marked = False

    def mark(self):
        """Record the point after encode on the current stream (no-op on CPU)."""
        import torch
        if self.stream is not None:
            self.event.record(torch.cuda.current_stream(self.gathered.device))
            self._marked = True

    def start(self, meta, maps):
        import torch
        if self.stream is None:
            pack_records(meta, maps, out=self.record)
            gather_records(self.record, self.group, out=self.gathered)
            return
        if self._marked:
            self.stream.wait_event(self.event)
            self._marked = False
        else:
            self.stream.wait_stream(torch.cuda.current_stream(meta.device))
        with torch.cuda.stream(self.stream):
            pack_records(meta, maps, out=self.record)
            gather_records(self.record, self.group, out=self.gathered)

    def join(self):
        import torch
        if self.stream is not None:
            torch.cuda.current_stream(self.gathered.device).wait_stream(self.stream)
        return self.gathered
