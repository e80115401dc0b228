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


def _pee_records(lo, hi, lm_words, heavy=()):
    """codec_pee_meta rows with end = 37 * g + 5 (g = global slice id); the location map of
    slice g has bits 3g+1 and 5g+2 set (a few overflow candidates, sparse records) -- or, for
    g in `heavy`, every third candidate up to `end` (an overflow-heavy slice, e.g. uniform
    u16 data, whose record goes dense) -- and garbage (-7) past `end`, which the exchange
    must drop.  lm_count = the map's popcount, as the embed writes it."""
    import numpy as np
    B = hi - lo
    meta = torch.zeros((B, _lib.PEE_META_BYTES), dtype=torch.uint8)
    lm = torch.full((B, lm_words), -7, dtype=torch.int64)
    for i in range(B):
        g = lo + i
        end = 37 * g + 5
        bits = np.zeros(64 * lm_words, dtype=np.uint8)
        if g in heavy:
            bits[0: end + 1: 3] = 1
        else:
            bits[[3 * g + 1, 5 * g + 2]] = 1
        bits[end + 1:] = 0
        nw = (end + 1 + 63) // 64
        words = np.packbits(bits, bitorder="little").view(np.int64)
        lm[i, :nw] = torch.from_numpy(words[:nw].copy())
        if (end + 1) % 64:                       # garbage past `end` inside its last word too
            lm[i, nw - 1] |= torch.tensor(-1 << ((end + 1) % 64), dtype=torch.int64)
        m = meta[i].view(torch.int32)
        m[0], m[2], m[3], m[4], m[9] = 2, 1000 + g, end, 64 * lm_words, int(bits.sum())
    return meta, lm


def _want_map(g, lm_words, heavy=()):
    """Slice g's map as _pee_records defines it, dense, zero past `end`."""
    import numpy as np
    end = 37 * g + 5
    bits = np.zeros(64 * lm_words, dtype=np.uint8)
    if g in heavy:
        bits[0: end + 1: 3] = 1
    else:
        bits[[3 * g + 1, 5 * g + 2]] = 1
    bits[end + 1:] = 0
    return torch.from_numpy(np.packbits(bits, bitorder="little").view(np.int64).copy())


def _want_width(gs, lm_words, heavy=()):
    """max over slices of min(ceil(popcount / 2), ceil((end + 1) / 64)), at least 1."""
    w = 1
    for g in gs:
        cnt = int(sum(bin(int(x) & (2**64 - 1)).count("1") for x in _want_map(g, lm_words, heavy)))
        w = max(w, min((cnt + 1) // 2, (37 * g + 5 + 64) // 64))
    return w


def test_pee_records_pack_unpack_cpu():
    """Sparse and dense records (codec_pee_pack_records' rule) round-trip every map exactly,
    and the width rule picks the shorter form per slice."""
    lm_words = 16
    heavy = (5,)
    meta, lm = _pee_records(0, 8, lm_words, heavy)
    need = int(D.record_width_needed(meta, lm_words))
    # sparse slices need ceil(2 / 2) = 1 word; slice 5 (end 190, 64 set bits) needs min(32, 3) = 3
    assert need == 3
    for width in (need, need + 4):
        rec = D.pack_pee_records(meta, lm, width)
        assert tuple(rec.shape) == (8, D.PEE_META_WORDS + width)
        m2, l2 = D.unpack_pee_records(rec, lm_words)
        assert torch.equal(m2, meta)
        for g in range(8):
            assert torch.equal(l2[g], _want_map(g, lm_words, heavy)), (width, g)
        assert torch.equal(l2, D.map_prefix(meta, lm, lm_words))
    # too narrow a width cuts the heavy slice's map (what overflows() counts)
    rec = D.pack_pee_records(meta, lm, 1)
    _m, l1 = D.unpack_pee_records(rec, lm_words)
    assert not torch.equal(l1[5], _want_map(5, lm_words, heavy))


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
    # ---- MED-PEE records: meta + the map, sparse or dense (slice 2 is overflow-heavy)
    lm_words = 16
    heavy = (2,)
    pmeta, lm = _pee_records(lo, hi, lm_words, heavy)
    px = D.PeeRecordExchange(B, world, "cpu", n_total=n_slices)
    px.mark()
    px.start(pmeta, lm)
    gmeta, glm = px.join()
    end_max = 37 * (n_slices - 1) + 5
    ok &= px.width == _want_width(range(n_slices), lm_words, heavy)
    ok &= tuple(gmeta.shape) == (n_slices, _lib.PEE_META_BYTES)
    ok &= tuple(glm.shape) == (n_slices, (end_max + 1 + 63) // 64)
    for g in range(n_slices):
        m = gmeta[g].contiguous().view(torch.int32)
        ok &= int(m[2]) == 1000 + g and int(m[3]) == 37 * g + 5
        ok &= torch.equal(glm[g], _want_map(g, lm_words, heavy)[: glm.shape[1]])
    own = px.own_rows(rank)
    ok &= torch.equal(own, D.pack_pee_records(pmeta, lm, px.width))
    ok &= px.overflows() == 0
    # ---- a later step whose maps need more: the carried width is too narrow for that
    # gather (the device counts it); join() is exact anyway (it re-gathers at the needed
    # width), and the following step adopts that width without any host read
    w0 = px.width
    heavy2 = tuple(range(n_slices))                                  # every slice overflow-heavy
    pmeta2, lm2 = _pee_records(lo, hi, lm_words, heavy2)
    w1 = _want_width(range(n_slices), lm_words, heavy2)
    px.start(pmeta2, lm2)
    ok &= px.overflows() == int(w1 > w0) and px.width == w0
    rec_cut = px.join_records()                                      # the benchmark's unverified view
    ok &= rec_cut.shape[1] == D.PEE_META_WORDS + w0
    gmeta2, glm2 = px.join()                                         # exact by default
    ok &= px.overflows() == 0 and px.width == w1
    for g in range(n_slices):
        ok &= torch.equal(glm2[g], _want_map(g, lm_words, heavy2)[: glm2.shape[1]])
    px.start(pmeta2, lm2)
    ok &= px.width == w1 and px.overflows() == 0 and px.verify() is False
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


@pytest.mark.parametrize("world,n_slices", [(4, 11), (8, 19)])
def test_exchanges_gloo_more_ranks(world, n_slices):
    """The same exchanges rehearsed at 4 and 8 ranks (the driver's scaling run uses up to 8
    GPUs), uneven shards (11 = 3 + 3 + 3 + 2; 19 over 8 ranks: three of 3, five of 2)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_slices, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=180) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(ok for _r, ok in res), res


def _ranks_worker(rank, world, port, same_device, q):
    """bench.gather_rank_records over gloo: every rank gets every record in rank order; with
    the RCCL check on, two ranks naming one (host, PCI) device is an error."""
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    # "partitions": one PCI address, distinct device UUIDs (compute partitions of one package)
    pci = "0000:%02x:00" % (rank if same_device == "distinct" else 0)
    uuid = "%032x" % (rank if same_device == "partitions" else 7)
    rec = {"rank": rank, "host": "h", "pci": pci, "uuid": uuid, "ms_per_step": 1.0 + rank}
    out = bench.gather_rank_records(torch, dist, world, rec, "gloo")
    ok = [r["rank"] for r in out] == list(range(world)) and out[rank] == rec
    shared = same_device == "shared"
    try:
        bench.gather_rank_records(torch, dist, world, rec, "nccl")
        ok &= not shared
    except RuntimeError as e:
        ok &= shared and "distinct devices" in str(e)
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("same_device", ["distinct", "shared", "partitions"])
def test_rank_records_gathered_and_checked(same_device):
    """the per-rank records of the N > 1 bench line arrive in rank order,
    and over RCCL a shared device is refused -- a device being (host, PCI address, UUID), so
    compute partitions of one package (one PCI address, distinct UUIDs) are distinct."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ranks_worker, args=(r, world, port, same_device, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=120) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(ok for _r, ok in res), res
