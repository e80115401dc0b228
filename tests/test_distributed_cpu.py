"""world_size-2 gloo test of the multi-GPU bookkeeping (sharding + record all-gather).
The HIP kernels are not involved (no GPU here); meta/maps are synthetic records."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from codec_tcc_amd import _lib, distributed as D


def test_shard_range_covers_everything():
    for n in (0, 1, 7, 256, 2048, 2049):
        for w in (1, 2, 3, 8):
            spans = [D.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_pack_unpack_roundtrip():
    B, mw = 5, 3
    meta = torch.randint(0, 256, (B, _lib.META_BYTES), dtype=torch.uint8)
    maps = torch.randint(-2**62, 2**62, (B, mw), dtype=torch.int64)
    rec = D.pack_records(meta, maps)
    assert rec.shape == (B, D.record_words(mw))
    m2, p2 = D.unpack_records(rec, mw)
    assert torch.equal(m2, meta) and torch.equal(p2, maps)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_slices, mw, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = D.shard_range(n_slices, world, rank)
    B = hi - lo
    # records whose content encodes the global slice id, so placement can be checked
    meta = torch.zeros((B, _lib.META_BYTES), dtype=torch.uint8)
    for i in range(B):
        meta[i, :4] = torch.tensor(list(int(lo + i).to_bytes(4, "little")), dtype=torch.uint8)
    maps = torch.arange(lo * mw, hi * mw, dtype=torch.int64).view(B, mw)
    rec = D.pack_records(meta, maps)
    allrec = D.gather_records(rec)
    gm, gp = D.unpack_records(allrec, mw)
    ok = True
    for g in range(n_slices):
        ok &= int.from_bytes(bytes(gm[g, :4].tolist()), "little") == g
        ok &= torch.equal(gp[g], torch.arange(g * mw, (g + 1) * mw, dtype=torch.int64))
    # the overlapped exchange (CPU tensors: synchronous) yields the same records
    xch = D.RecordExchange(B, mw, world, "cpu")
    xch.start(meta, maps)
    ok &= torch.equal(xch.join(), allrec)
    q.put((rank, bool(ok), tuple(allrec.shape)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_records_gloo(world):
    n_slices, mw = 8, 5            # equal shards (all_gather_into_tensor needs equal sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_slices, mw, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _r, ok, _s in res), res
    assert all(s == (n_slices, D.record_words(mw)) for _r, _ok, s in res)
