"""world_size-2 gloo tests of the multi-GPU bookkeeping (sharding + record all-gathers).
The HIP kernels are not involved (no GPU here); meta/maps are synthetic records whose
content encodes the global slice id, so their placement after the gather can be checked."""
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
            assert max(sizes) <= D.shard_rows(n, w)


def test_valid_rows_uneven():
    # 2049 slices over 8 ranks: 257 rows per rank, the last 7 ranks have one padding row
    idx = D.valid_rows(2049, 8)
    assert len(idx) == 2049 and idx == sorted(idx)
    assert D.shard_rows(2049, 8) == 257
    assert idx[256] == 256 and idx[257] == 257 + 0 and idx[-1] == 7 * 257 + 255


def test_pack_unpack_roundtrip():
    B, mw = 5, 3
    meta = torch.randint(0, 256, (B, _lib.META_BYTES), dtype=torch.uint8)
    maps = torch.randint(-2**62, 2**62, (B, mw), dtype=torch.int64)
    rec = D.pack_records(meta, maps)
    assert rec.shape == (B, D.record_words(mw))
    m2, p2 = D.unpack_records(rec, mw)
    assert torch.equal(m2, meta) and torch.equal(p2, maps)
    wide = torch.full((B, D.record_words(mw + 2)), -1, dtype=torch.int64)
    D.pack_records(meta, maps, out=wide)                 # job-wide width: zero tail
    m3, p3 = D.unpack_records(wide, mw + 2)
    assert torch.equal(m3, meta) and torch.equal(p3[:, :mw], maps) and not p3[:, mw:].any()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lsb_records(lo, hi, mw):
    B = hi - lo
    meta = torch.zeros((B, _lib.META_BYTES), dtype=torch.uint8)
    for i in range(B):
        meta[i, :4] = torch.tensor(list(int(lo + i).to_bytes(4, "little")), dtype=torch.uint8)
    maps = torch.arange(lo * mw, hi * mw, dtype=torch.int64).view(B, mw) if B else torch.zeros((0, mw), dtype=torch.int64)
    return meta, maps


def _pee_records(lo, hi, lm_words):
    """codec_pee_meta rows with end = 37 * g + 5 (g = global slice id) and location maps
    whose words before the end carry g; words past `end` are garbage the exchange must drop."""
    B = hi - lo
    meta = torch.zeros((B, _lib.PEE_META_BYTES), dtype=torch.uint8)
    lm = torch.full((B, lm_words), -7, dtype=torch.int64)
    for i in range(B):
        g = lo + i
        m = meta[i].view(torch.int32)
        m[0], m[2], m[3], m[4] = 2, 1000 + g, 37 * g + 5, 64 * lm_words
        nw = (37 * g + 5 + 1 + 63) // 64
        lm[i, :nw] = torch.arange(nw, dtype=torch.int64) * 1000 + g
    return meta, lm


def _worker(rank, world, port, n_slices, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = D.shard_range(n_slices, world, rank)
    B = hi - lo
    ok = True
    # ---- LSB records; the map width differs per rank (payload lengths differ)
    mw = 5 if rank == 0 else 3
    meta, maps = _lsb_records(lo, hi, mw)
    xch = D.RecordExchange(B, mw, world, "cpu", n_total=n_slices)
    xch.start(meta, maps)
    allrec = xch.join()
    ok &= tuple(allrec.shape) == (n_slices, D.record_words(5))
    gm, gp = D.unpack_records(allrec, 5)
    for g in range(n_slices):
        r = next(r for r in range(world) if D.shard_range(n_slices, world, r)[0] <= g < D.shard_range(n_slices, world, r)[1])
        w = 5 if r == 0 else 3
        ok &= int.from_bytes(bytes(gm[g, :4].tolist()), "little") == g
        ok &= torch.equal(gp[g, :w], torch.arange(g * w, (g + 1) * w, dtype=torch.int64))
        ok &= not gp[g, w:].any()
    ok &= torch.equal(D.pack_records(meta, maps, out=torch.zeros((B, D.record_words(5)), dtype=torch.int64)),
                      xch.own_rows(rank))
    # ---- MED-PEE records: metas, then location-map prefixes up to the job's largest end
    lm_words = 16
    pmeta, lm = _pee_records(lo, hi, lm_words)
    px = D.PeeRecordExchange(B, world, "cpu", n_total=n_slices)
    px.mark()
    px.start(pmeta, lm)
    gmeta, glm = px.join()
    end_max = 37 * (n_slices - 1) + 5
    ok &= px.lm_words == (end_max + 1 + 63) // 64
    ok &= tuple(gmeta.shape) == (n_slices, _lib.PEE_META_BYTES) and tuple(glm.shape) == (n_slices, px.lm_words)
    for g in range(n_slices):
        m = gmeta[g].contiguous().view(torch.int32)
        ok &= int(m[2]) == 1000 + g and int(m[3]) == 37 * g + 5
        nw = (37 * g + 5 + 1 + 63) // 64
        ok &= torch.equal(glm[g, :nw], torch.arange(nw, dtype=torch.int64) * 1000 + g)
    om, ol = px.own_rows(rank)
    ok &= torch.equal(om.contiguous().view(torch.uint8)[:, : _lib.PEE_META_BYTES], pmeta)
    # words past each slice's own end were garbage (-7): the gathered rows carry zeros there
    for i in range(B):
        nw = (37 * (lo + i) + 5 + 1 + 63) // 64
        ok &= torch.equal(ol[i, :nw], lm[i, :nw]) and not ol[i, nw:].any()
    ok &= px.overflows() == 0
    # ---- a later step whose maps are longer: the carried width is too narrow for that
    # gather (the device counts it), verify() re-gathers it at the needed width, and the
    # following step adopts that width without any host read
    w0 = px.lm_words
    pmeta2, lm2 = _pee_records(lo, hi, lm_words)
    for i in range(B):
        pmeta2[i].view(torch.int32)[3] = 64 * (w0 + 1) + i          # end -> w0 + 2 words
        lm2[i, : w0 + 2] = torch.arange(w0 + 2, dtype=torch.int64) + 100 * (lo + i)
    px.start(pmeta2, lm2)
    ok &= px.overflows() == 1 and px.lm_words == w0
    ok &= px.verify() is True and px.overflows() == 0 and px.lm_words == w0 + 2
    gmeta2, glm2 = px.join()
    for g in range(n_slices):
        ok &= torch.equal(glm2[g, : w0 + 2], torch.arange(w0 + 2, dtype=torch.int64) + 100 * g)
    px.start(pmeta2, lm2)
    ok &= px.lm_words == w0 + 2 and px.overflows() == 0 and px.verify() is False
    # ---- the plain gather helper with equal shards
    rec = D.pack_records(*_lsb_records(lo, hi, 4))
    ok &= D.gather_records(rec, rows=D.shard_rows(n_slices, world)).shape[0] == world * D.shard_rows(n_slices, world)
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_slices", [8, 5, 3])
def test_exchanges_gloo_world2(n_slices):
    """Even (8) and uneven (5 = 3 + 2, 3 = 2 + 1) shards, for both record kinds."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_slices, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _r, ok in res), res
