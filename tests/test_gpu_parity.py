"""HIP path vs the reference (golden vectors) and vs the oracle, bit-exact.  Runs on the
MI355X box (`pytest -m gpu`); every call goes through the C ABI in libcodec_hip.so."""
import hashlib

import numpy as np
import pytest

import golden_io
from codec_tcc_amd import Codec, _lib, framing, synth
from codec_tcc_amd import codec as K
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CASES = [c for c in golden_io.cases() if str(c["embedder"]) in ("hybrid", "multi")]


def _run_case(case, all_mi=True, beta=None):
    cover = case["cover"]
    h, w = cover.shape
    nb = int(case["nbits"])
    nbits = None if nb < 0 else nb
    beta = float(case["beta"]) if beta is None else beta
    codec = Codec(1, h, w, dtype=str(cover.dtype), beta=beta, block=int(case["sb"]),
                  align=bool(case["align"]), mode=str(case["embedder"]), nbits=nbits, all_mi=all_mi)
    bitstr = str(case["bits"])
    bits = (np.frombuffer(bitstr.encode(), np.uint8) - 48) if bitstr else np.zeros(0, np.uint8)
    enc = codec.encode(torch.from_numpy(cover[None].copy()).cuda(), [bits])
    torch.cuda.synchronize()
    return codec, enc


@pytest.fixture(params=["split", "waves", "waves_full", "block", "fused"])
def decide_path(request, monkeypatch):
    """k_decide's split decision (default for small batches: one plane workgroup per MI
    plane), its one-workgroup wave-parallel MI path (CODEC_DECIDE_SPLIT=0; the default for
    big batches when the joint orders fit in LDS) and the block-sequential one
    (CODEC_DECIDE_WAVES=0; also what large-m slices use).  The block variant also runs
    codec_encode unfused (codec_plan then the separate k_embed launch).  "fused": the scan,
    decision and embed in one launch (k_scan_decide, CODEC_FUSED_DECIDE=2 forces it on these
    one-slice batches; cases it does not take -- uint8, other block sizes, edge blocks -- run
    the separate kernels).  "waves" runs the lean k_decide (guard-band fallbacks on the block
    path) unless all_mi asks for every exact value; "waves_full" keeps the wave-parallel exact
    rounds for the fallbacks as well (CODEC_DECIDE_LEAN=0)."""
    if request.param == "fused":
        monkeypatch.setenv("CODEC_FUSED_DECIDE", "2")
    if request.param == "split":   # plane workgroups also without all_mi (default: all_mi only)
        monkeypatch.setenv("CODEC_DECIDE_SPLIT", "2")
    if request.param in ("waves", "waves_full"):
        monkeypatch.setenv("CODEC_DECIDE_SPLIT", "0")
    if request.param == "waves_full":   # the k_decide instantiation with the wave-parallel exact
        monkeypatch.setenv("CODEC_DECIDE_LEAN", "0")   # rounds also without all_mi (guard fallbacks)
    if request.param == "block":
        monkeypatch.setenv("CODEC_DECIDE_WAVES", "0")
        monkeypatch.setenv("CODEC_FUSED_EMBED", "0")
    return request.param


def _ref_loop(mis, entropy, beta):
    """The reference's decision loop (codec.py:580-593) run on the reference's own float64
    MI values and entropy (the golden tables): s and cumulative_info."""
    tg = beta * entropy
    c = 0.0
    for i, mi in enumerate(mis):
        c += mi
        if c >= tg:
            return i + 1, c
    return 1, c


def _ref_evaluated(mis, entropy, beta):
    """How many planes the reference's loop evaluates (all of them when it never breaks)."""
    tg = beta * entropy
    c = 0.0
    for i, mi in enumerate(mis):
        c += mi
        if c >= tg:
            return i + 1
    return len(mis)


@pytest.mark.parametrize("all_mi", [True, False], ids=["exact_mi", "guarded"])
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_case(case, decide_path, all_mi):
    """all_mi: every plane's MI by the numpy-order sums (bit-exact); guarded: the default
    guard-banded decision -- same s and outputs, mi[] = H(X) of the evaluated planes."""
    codec, enc = _run_case(case, all_mi=all_mi)
    m = enc.records()[0]
    s = int(case["s"])
    assert m.status == 0
    assert m.s == s
    assert [m.perm[j] for j in range(s)] == list(case["perm"])
    assert [m.sizes[p] for p in range(s)] == list(case["sizes"])
    assert m.total_used == int(case["total_used"])
    # bit-exact float64 information values (calculate_entropy / calculate_mutual_information)
    assert m.entropy == float(case["entropy"])
    nb = len(case["mi"])
    if all_mi or int(case.get("fixed_s", 0)) > 0:
        assert [m.mi[i] for i in range(nb)] == list(case["mi"])
        assert not (m.flags & (_lib.FLAG_INFO_FAST | _lib.FLAG_GUARD_FALLBACK))
    elif m.flags & _lib.FLAG_INFO_FAST:
        assert not (m.flags & _lib.FLAG_GUARD_FALLBACK)
        ev = _ref_evaluated(list(case["mi"]), float(case["entropy"]), float(case["beta"]))
        for i in range(nb):   # H(X) vs the reference's h_x + h_y - h_xy: rounding only
            assert abs(m.mi[i] - float(case["mi"][i])) <= 1e-12 if i < ev else m.mi[i] == 0.0, i
    else:   # inside the guard band: the exact sums decided
        assert m.flags & _lib.FLAG_GUARD_FALLBACK
        ev = _ref_evaluated(list(case["mi"]), float(case["entropy"]), float(case["beta"]))
        assert [m.mi[i] for i in range(ev)] == list(case["mi"])[:ev]
    # stego pixels
    exp = golden_io.stego(case)
    got = enc.stego.cpu().numpy()[0]
    assert got.dtype == exp.dtype
    np.testing.assert_array_equal(got, exp)
    # dense reference bitmaps
    dense = codec.expand_maps(enc.maps, enc.meta, map_words=enc.payloads.map_words).cpu().numpy()[0]
    np.testing.assert_array_equal(dense[:s], golden_io.dense_bitmaps(case))
    assert not dense[s:].any()
    # the reference's own decode_message output (lossy), bit-exact
    if True:
        dec_codec = K._codec_for(tuple(enc.stego.shape), str(enc.stego.dtype), **K._codec_kw(enc))
        b, cnt = dec_codec.decode_ref_compat_bits(enc.stego, enc.maps, enc.meta, map_words=enc.payloads.map_words)
        n = int(cnt.cpu()[0])
        txt = framing.bits_to_bytes_msb(b.cpu().numpy()[0, :n]).decode("utf-8", errors="replace")
        assert txt == golden_io.decoded(case)
    # true extraction: payload in message order + cover restored
    payload, cover = K.decode(enc)
    exp_bits = str(case["bits"])
    sizes = list(case["sizes"])
    npx = case["cover"].size
    tiling = min(sizes) >= 0 and all(x <= npx for x in sizes) and str(case["embedder"]) == "hybrid"
    if tiling:
        assert framing.bits_to_str(payload[0]) == exp_bits
    keep = (1 << (8 * enc.stego.element_size())) - 1
    nbits = int(case["nbits"])
    if nbits > 0:
        keep = (1 << nbits) - 1
    np.testing.assert_array_equal(cover.cpu().numpy()[0], (case["cover"].astype(np.uint32) & keep).astype(exp.dtype))


@pytest.mark.parametrize("kind,h,w,bsz", [("ct12", 512, 512, 5), ("u16", 256, 320, 3), ("u8", 200, 96, 4),
                                          ("ct12", 120, 136, 3)])
def test_batch_vs_oracle(kind, h, w, bsz, decide_path):
    gen = synth.GENERATORS[kind]
    covers = np.stack([gen(h, w, 100 + i) for i in range(bsz)])
    msgs = [synth.payload(64 + 37 * i, i) for i in range(bsz)]
    codec = Codec(bsz, h, w, dtype=str(covers.dtype), beta=0.4, block=16)
    enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
    torch.cuda.synchronize()
    stego = enc.stego.cpu().numpy()
    recs = enc.records()
    bits, cover = K.decode(enc)
    refs = K.decode_ref_compat(enc)
    for i in range(bsz):
        mb = R.message_to_bits(msgs[i])
        exp = R.encode_slice(covers[i], mb, beta=0.4, sb=16)
        assert recs[i].s == exp["s"]
        assert recs[i].start_offset == exp["start_offset"]
        np.testing.assert_array_equal(stego[i], exp["stego"])
        assert framing.bits_to_str(bits[i]) == mb
        assert refs[i] == R.decode_slice(exp["stego"], exp["bitmaps"], exp["s"], exp["segments_lengths"],
                                         exp["segment_indices"])
    np.testing.assert_array_equal(cover.cpu().numpy(), covers)


@pytest.mark.parametrize("kat", golden_io.kat2048(), ids=lambda k: f"{k['kind']}{k['seed']}b{k['beta']}")
def test_kat_2048(kat, decide_path):
    """Full-size (2048^2) known answers from the reference, as sha256 digests."""
    img = synth.GENERATORS[kat["kind"]](kat["h"], kat["w"], kat["seed"])
    assert hashlib.sha256(img.tobytes()).hexdigest() == kat["cover_sha256"]
    msg = synth.payload(kat["payload_chars"], kat["payload_seed"])
    codec = Codec(1, kat["h"], kat["w"], dtype="uint16", beta=kat["beta"], block=16)
    enc = codec.encode(torch.from_numpy(img[None].copy()).cuda(), [msg])
    m = enc.records()[0]
    assert m.s == kat["s"]
    assert [m.perm[j] for j in range(m.s)] == kat["perm"]
    assert [m.sizes[p] for p in range(m.s)] == kat["sizes"]
    assert hashlib.sha256(enc.stego.cpu().numpy().tobytes()).hexdigest() == kat["stego_sha256"]
    dense = codec.expand_maps(enc.maps, enc.meta, map_words=enc.payloads.map_words).cpu().numpy()[0, : m.s]
    assert hashlib.sha256(dense.tobytes()).hexdigest() == kat["bitmaps_sha256"]
    txt = K.decode_ref_compat(enc)[0]
    assert len(txt) == kat["decoded_len"]
    assert hashlib.sha256(txt.encode("utf-8")).hexdigest() == kat["decoded_sha256"]
    bits, cover = K.decode(enc)
    assert framing.bits_to_str(bits[0]) == R.message_to_bits(msg)
    np.testing.assert_array_equal(cover.cpu().numpy()[0], img)


@pytest.mark.parametrize("sweep", ["0", "1"])
def test_roundtrip_full_size_batch(monkeypatch, sweep):
    """256-slice-class property check at bench size, smaller batch: encode->decode is the
    identity on cover and payload (size-independent property); both scan sweeps (this
    64 MiB batch would take the band sweep by default)."""
    monkeypatch.setenv("CODEC_SCAN_KIND", sweep)
    B, H, W = 8, 2048, 2048
    covers = torch.stack([torch.from_numpy(synth.ct12(H, W, i)) for i in range(B)]).cuda()
    msgs = [synth.payload(1024, 7 + i) for i in range(B)]
    codec = Codec(B, H, W, dtype="uint16", beta=0.4, block=16)
    enc = codec.encode(covers, msgs)
    bits, cover = K.decode(enc)
    assert torch.equal(cover.view(torch.int16), covers.view(torch.int16))
    for i in range(B):
        assert framing.bits_to_str(bits[i]) == R.message_to_bits(msgs[i])
    # stego differs from cover only in the payload windows
    diff = (enc.stego.view(torch.int16) != covers.view(torch.int16)).sum().item()
    assert 0 < diff <= sum(len(R.message_to_bits(m)) for m in msgs)


def test_shape_errors():
    codec = Codec(2, 64, 64, dtype="uint16")
    with pytest.raises(ValueError):
        codec.encode(torch.zeros((1, 64, 64), dtype=torch.uint16, device="cuda"), ["a"])
    with pytest.raises(TypeError):
        codec.encode(torch.zeros((2, 64, 64), dtype=torch.uint8, device="cuda"), ["a", "b"])


INPLACE = [c for c in CASES if int(c["nbits"]) < 0 or int(c["nbits"]) > 8 * c["cover"].dtype.itemsize - 8]


@pytest.mark.parametrize("case", INPLACE, ids=[c["name"] for c in INPLACE])
def test_inplace_matches_out_of_place(case):
    """stego == cover (codec_plan reads only, codec_embed patches the windows) and
    cover_out == stego (only the window pixels are XOR-ed back) give the out-of-place
    results bit for bit."""
    codec, enc = _run_case(case)
    cover = case["cover"]
    bitstr = str(case["bits"])
    bits = (np.frombuffer(bitstr.encode(), np.uint8) - 48) if bitstr else np.zeros(0, np.uint8)
    buf = torch.from_numpy(cover[None].copy()).cuda()
    enc2 = codec.encode(buf, [bits], stego=buf)
    assert enc2.stego.data_ptr() == buf.data_ptr()
    np.testing.assert_array_equal(buf.cpu().numpy()[0], golden_io.stego(case))
    used = (enc.records()[0].total_used + 63) // 64   # words past the embedded bits are unspecified
    np.testing.assert_array_equal(enc2.maps.cpu().numpy()[:, :used], enc.maps.cpu().numpy()[:, :used])
    np.testing.assert_array_equal(enc2.meta.cpu().numpy(), enc.meta.cpu().numpy())
    pw, mw = enc.payloads.payload_words, enc.payloads.map_words
    words_a, cover_a = codec.decode(enc.stego, enc.maps, enc.meta, payload_words=pw, map_words=mw)
    words_b, cover_b = codec.decode(buf, enc2.maps, enc2.meta, payload_words=pw, map_words=mw, cover=buf)
    assert cover_b.data_ptr() == buf.data_ptr()
    np.testing.assert_array_equal(words_b.cpu().numpy(), words_a.cpu().numpy())
    np.testing.assert_array_equal(buf.cpu().numpy(), cover_a.cpu().numpy())


@pytest.mark.parametrize("kind,h,w,bsz,mode", [("ct12", 512, 512, 4, "hybrid"), ("u16", 256, 320, 3, "hybrid"),
                                               ("u8", 200, 96, 3, "hybrid"), ("ct12", 128, 128, 3, "multi"),
                                               ("ct12", 37, 53, 2, "hybrid")])
def test_inplace_batch_roundtrip(kind, h, w, bsz, mode, decide_path):
    gen = synth.GENERATORS[kind]
    covers = np.stack([gen(h, w, 300 + i) for i in range(bsz)])
    msgs = [synth.payload(40 + 53 * i, 11 + i) for i in range(bsz)]
    codec = Codec(bsz, h, w, dtype=str(covers.dtype), beta=0.4, block=16, mode=mode)
    ref = codec.encode(torch.from_numpy(covers).cuda(), msgs)
    buf = torch.from_numpy(covers.copy()).cuda()
    enc = codec.encode(buf, msgs, stego=buf)
    np.testing.assert_array_equal(buf.cpu().numpy(), ref.stego.cpu().numpy())
    pw, mw = enc.payloads.payload_words, enc.payloads.map_words
    words, _ = codec.decode(buf, enc.maps, enc.meta, payload_words=pw, map_words=mw, cover=buf)
    ref_words, _ = codec.decode(ref.stego, ref.maps, ref.meta, payload_words=pw, map_words=mw)
    np.testing.assert_array_equal(words.cpu().numpy(), ref_words.cpu().numpy())
    np.testing.assert_array_equal(buf.cpu().numpy(), covers)


SWEEPS = [("0", None), ("1", None), ("1", "1"), ("1", "7"), ("1", "100000")]


@pytest.mark.parametrize("kind,h,w,sb", [("ct12", 512, 512, 16), ("ct12", 200, 136, 16), ("u16", 96, 264, 8),
                                         ("u8", 130, 72, 32), ("ct12", 256, 192, 64), ("u16", 64, 2048, 16)])
@pytest.mark.parametrize("sweep,wgs", SWEEPS, ids=[f"kind{a}-wgs{b}" for a, b in SWEEPS])
def test_scan_sweeps_agree_with_oracle(monkeypatch, kind, h, w, sb, sweep, wgs):
    """Both scan sweeps (column-band k_scan_fast, row-major k_scan_rows) at several
    workgroup-region sizes (whole slice per workgroup ... one band per workgroup) give the
    oracle's s, start offset and stego, including ragged last bands, W % SB != 0 (no lane
    grouping of block counts) and partial last iterations."""
    monkeypatch.setenv("CODEC_SCAN_KIND", sweep)
    monkeypatch.setenv("CODEC_SCAN_READ_KIND", sweep)
    if wgs is not None:
        monkeypatch.setenv("CODEC_SCAN_ROWS_WGS", wgs)
    gen = synth.GENERATORS[kind]
    bsz = 3
    covers = np.stack([gen(h, w, 500 + i) for i in range(bsz)])
    msgs = [synth.payload(90 + 31 * i, 40 + i) for i in range(bsz)]
    codec = Codec(bsz, h, w, dtype=str(covers.dtype), beta=0.4, block=sb)
    enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
    stego = enc.stego.cpu().numpy()
    recs = enc.records()
    for i in range(bsz):
        exp = R.encode_slice(covers[i], R.message_to_bits(msgs[i]), beta=0.4, sb=sb)
        assert recs[i].s == exp["s"]
        assert recs[i].start_offset == exp["start_offset"]
        np.testing.assert_array_equal(stego[i], exp["stego"])
    buf = torch.from_numpy(covers.copy()).cuda()          # read-only sweep (in place)
    enc2 = codec.encode(buf, msgs, stego=buf)
    np.testing.assert_array_equal(buf.cpu().numpy(), stego)
    assert [r.start_offset for r in enc2.records()] == [r.start_offset for r in recs]


@pytest.mark.parametrize("kind,h,w,chars", [("ct12", 512, 512, 3000), ("u8", 300, 200, 2600), ("ct12", 5, 24, 4),
                                            ("ct12", 40, 8, 9), ("u16", 64, 2048, 2100)])
def test_long_payloads_and_tiny_shapes(kind, h, w, chars, decide_path):
    """Payloads longer than one 8192-bit round of the fused embed / gather loops, and shapes
    with no full 16x16 block (H or W < 16): bit-exact vs the oracle, exact recovery."""
    gen = synth.GENERATORS[kind]
    bsz = 2
    covers = np.stack([gen(h, w, 900 + i) for i in range(bsz)])
    msgs = [synth.payload(chars - 3 * i, 60 + i) for i in range(bsz)]
    codec = Codec(bsz, h, w, dtype=str(covers.dtype), beta=0.4, block=16)
    enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
    stego = enc.stego.cpu().numpy()
    recs = enc.records()
    bits, cover = K.decode(enc)
    for i in range(bsz):
        mb = R.message_to_bits(msgs[i])
        exp = R.encode_slice(covers[i], mb, beta=0.4, sb=16)
        assert recs[i].s == exp["s"] and recs[i].start_offset == exp["start_offset"]
        np.testing.assert_array_equal(stego[i], exp["stego"])
        n = sum(exp["segments_lengths"]) if min(exp["segments_lengths"]) >= 0 else None
        if n == len(mb) and max(exp["segments_lengths"]) <= h * w:
            assert framing.bits_to_str(bits[i]) == mb
    np.testing.assert_array_equal(cover.cpu().numpy(), covers)


@pytest.mark.parametrize("sweep", ["0", "1"])
def test_histogram_wraps_on_flat_slices(monkeypatch, sweep):
    """Flat regions put > 65 535 pixels of one value into one workgroup's 16-bit LDS bin
    halves (and equal-neighbour runs into single adds): the exact wrap bookkeeping must still
    give the oracle's entropy / MI decisions, offsets and stego."""
    monkeypatch.setenv("CODEC_SCAN_KIND", sweep)
    h = w = 1024
    a = np.full((h, w), 1234, np.uint16)                       # constant slice
    b = synth.ct12(h, w, 5).copy()
    b[:, : w // 2] = 0                                         # half black (air), half tissue
    c = synth.ct12(h, w, 6).copy()
    c[::2, ::2] = 4095                                         # a dense saturated lattice
    covers = np.stack([a, b, c])
    msgs = [synth.payload(300 + 50 * i, 80 + i) for i in range(3)]
    codec = Codec(3, h, w, dtype="uint16", beta=0.4, block=16, all_mi=True)
    enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
    stego = enc.stego.cpu().numpy()
    recs = enc.records()
    for i in range(3):
        exp = R.encode_slice(covers[i], R.message_to_bits(msgs[i]), beta=0.4, sb=16)
        assert recs[i].s == exp["s"] and recs[i].start_offset == exp["start_offset"]
        np.testing.assert_array_equal(stego[i], exp["stego"])
        assert recs[i].entropy == R.entropy(covers[i])


def _wide_cover(kind, h, w, seed):
    rng = np.random.default_rng(seed)
    if kind == "dense":                       # every 16-bit value present, small counts
        return rng.integers(0, 65536, (h, w)).astype(np.uint16)
    if kind == "sparse":                      # ~12k distinct values spread over the range
        vals = np.sort(rng.choice(65536, 12000, replace=False)).astype(np.uint16)
        return vals[rng.integers(0, vals.size, (h, w))]
    if kind == "bigcounts":                   # half the pixels on 10 values (counts >> 1024)
        img = rng.integers(0, 65536, (h, w)).astype(np.uint16)
        mask = rng.random((h, w)) < 0.5
        img[mask] = rng.choice(np.array([0, 1, 7, 1000, 4095, 4096, 30000, 32768, 65534, 65535], np.uint16),
                               int(mask.sum()))
        return img
    if kind == "halfrange":                   # values < 32768 (Rp = 32768, 32 bins per thread)
        return rng.integers(0, 32768, (h, w)).astype(np.uint16)
    raise ValueError(kind)


@pytest.mark.parametrize("kind,h,w", [("dense", 512, 512), ("sparse", 384, 512), ("bigcounts", 512, 512),
                                      ("halfrange", 300, 700), ("dense", 97, 211)])
def test_wide_slices_information_exact(kind, h, w, decide_path):
    """Slices with too many distinct values for the wave path's LDS arena: k_decide's walk
    path (default) and the block path agree with numpy's entropy / MI bit for bit."""
    cover = _wide_cover(kind, h, w, 5)
    codec = Codec(1, h, w, dtype="uint16", beta=0.8, block=16, all_mi=True)
    enc = codec.encode(torch.from_numpy(cover[None].copy()).cuda(), [synth.payload(100, 1)])
    m = enc.records()[0]
    assert m.status == 0
    assert m.nonzero_bins == np.unique(cover).size
    assert m.entropy == R.entropy(cover)
    for i in range(16):
        assert m.mi[i] == R.mutual_information((cover >> i) & 1, cover), i
    exp = R.encode_slice(cover, R.message_to_bits(synth.payload(100, 1)), beta=0.8, sb=16)
    assert m.s == exp["s"]
    np.testing.assert_array_equal(enc.stego.cpu().numpy()[0], exp["stego"])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,kinds", [("uint16", ["u16", "ct12", "zero", "ct12", "u16"]),
                                         ("uint8", ["u8", "zero", "u8"])])
def test_workspace_reuse_stays_clean(dtype, kinds, monkeypatch):
    """codec_plan does not memset its workspace per call: k_decide clears the histogram
    bins, block key and OR word it consumed.  One Codec over batches of different value
    ranges (wide, narrow, constant zero, back to wide) must match the oracle on every call.
    One scan workgroup per slice, so the 262 144 zeros of a slice wrap the 16-bit LDS bin
    halves (the wrap fix-up writes bin 1, above Rp = 1)."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("CODEC_SCAN_WGS", "1")
    monkeypatch.setenv("CODEC_SCAN_ROWS_WGS", "1")
    B, H, W = 2, 512, 512
    codec = Codec(B, H, W, dtype=dtype, beta=0.4, block=16, device="cuda")
    for step, kind in enumerate(kinds):
        if kind == "zero":
            covers = np.zeros((B, H, W), dtype=dtype)
        else:
            covers = np.stack([synth.GENERATORS[kind](H, W, 60 + 7 * step + i) for i in range(B)]).astype(dtype)
        msgs = [synth.payload(200 + 30 * i, 90 + step + i) for i in range(B)]
        enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
        recs = enc.records()
        stego = enc.stego.cpu().numpy()
        for i in range(B):
            exp = R.encode_slice(covers[i], R.message_to_bits(msgs[i]), beta=0.4, sb=16)
            assert recs[i].s == exp["s"], (step, kind, i)
            assert recs[i].start_offset == exp["start_offset"], (step, kind, i)
            np.testing.assert_array_equal(stego[i], exp["stego"])


@pytest.mark.parametrize("restore", ["ss", "ss_copy_hull", "ss_d4", "ss_d16", "ss_late", "gs"])
@pytest.mark.parametrize("kind,h,w,bsz,chars", [("ct12", 512, 512, 5, 1024), ("u8", 256, 256, 3, 2500),
                                                ("u16", 256, 512, 2, 4000), ("ct12", 256, 256, 4, 3000)])
def test_restore_paths_vs_oracle(kind, h, w, bsz, chars, restore, monkeypatch):
    """codec_extract's out-of-place restore through the slice-serial pass (forced here, the
    default for batches of >= one slice per CU) -- "ss": k_restore_il (ring copy with the hull
    restored and the payload gathered inline from LDS-staged maps), "ss_copy_hull" and the
    depth / late-gather variants: k_restore_ss (ring copy, then the window-hull rewrite; gather
    first or last) -- and the grid-stride pass: payload bits and restored cover exact, stego vs
    the oracle; long payloads make windows wrap past the slice end."""
    monkeypatch.setenv("CODEC_RESTORE_SS", "0" if restore == "gs" else "1")
    if restore == "ss_copy_hull":
        monkeypatch.setenv("CODEC_RESTORE_IL", "0")
    if restore in ("ss_d4", "ss_d16"):   # ring depths other than the default 8 vectors per thread
        monkeypatch.setenv("CODEC_RESTORE_SS_DEPTH", restore[4:])
    if restore == "ss_late":             # payload gather after the copy instead of before it
        monkeypatch.setenv("CODEC_RESTORE_SS_GLATE", "1")
    gen = synth.GENERATORS[kind]
    covers = np.stack([gen(h, w, 300 + i) for i in range(bsz)])
    msgs = [synth.payload(chars - 17 * i, 60 + i) for i in range(bsz)]
    codec = Codec(bsz, h, w, dtype=str(covers.dtype), beta=0.4, block=16)
    enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
    recs = enc.records()
    bits, cover = K.decode(enc)
    stego = enc.stego.cpu().numpy()
    for i in range(bsz):
        mb = R.message_to_bits(msgs[i])
        exp = R.encode_slice(covers[i], mb, beta=0.4, sb=16)
        assert recs[i].s == exp["s"] and recs[i].start_offset == exp["start_offset"]
        np.testing.assert_array_equal(stego[i], exp["stego"])
        assert framing.bits_to_str(bits[i]) == mb
    np.testing.assert_array_equal(cover.cpu().numpy(), covers)


def test_split_decision_timeout_leaves_no_stale_slot(monkeypatch):
    """a split decision whose main workgroup gives up on a plane slot (status 2,
    CODEC_FLAG_DECIDE_TIMEOUT) must not leave a value behind for the next call.  With
    CODEC_DECIDE_DEBUG_LATE=1 plane 0 of slice 0 publishes only after the main workgroup
    abandoned its slot (and CODEC_DECIDE_SPINS=200 makes it give up early, possibly on other
    slots too); Codec.encode raises on the status by default.  The next normal call must
    then decide every slice exactly as before (same s, MI values, stego, maps)."""
    from codec_tcc_amd import _lib
    B, H, W = 2, 512, 512
    covers = torch.from_numpy(np.stack([synth.ct12(H, W, 90 + i) for i in range(B)])).cuda()
    msgs = [synth.payload(300, 40 + i) for i in range(B)]
    codec = Codec(B, H, W, dtype="uint16", beta=0.4, block=16, all_mi=True)
    ref = codec.encode(covers, msgs)
    rr = ref.records()
    assert all(r.status == 0 for r in rr)
    monkeypatch.setenv("CODEC_DEBUG", "1")               # the fault-injection knobs' master switch
    monkeypatch.setenv("CODEC_DECIDE_SPINS", "200")
    monkeypatch.setenv("CODEC_DECIDE_DEBUG_LATE", "1")
    with pytest.raises(RuntimeError, match="timed out"):
        codec.encode(covers, msgs)
    bad = codec.encode(covers, msgs, check=False).records()
    assert bad[0].status == 2 and (bad[0].flags & _lib.FLAG_DECIDE_TIMEOUT)
    monkeypatch.delenv("CODEC_DECIDE_SPINS")
    monkeypatch.delenv("CODEC_DECIDE_DEBUG_LATE")
    for _ in range(2):
        enc = codec.encode(covers, msgs)
        torch.cuda.synchronize()
        assert torch.equal(enc.meta, ref.meta)
        assert torch.equal(enc.stego.view(torch.int16), ref.stego.view(torch.int16))
        assert torch.equal(enc.maps, ref.maps)


@pytest.mark.parametrize("fused", [True, False])
def test_maps_fully_defined(fused, monkeypatch):
    """Every word of the location-map rows is written (zero past the bits used), whatever the
    output buffer held before -- the fused decision's embed and k_embed alike."""
    if not fused:
        monkeypatch.setenv("CODEC_FUSED_EMBED", "0")
    B, H, W = 2, 256, 256
    covers = torch.from_numpy(np.stack([synth.ct12(H, W, 60 + i) for i in range(B)])).cuda()
    msgs = [synth.payload(40, 3), synth.payload(400, 4)]   # short and long: many unused words
    codec = Codec(B, H, W, dtype="uint16", beta=0.4, block=16)
    pl = K.make_payloads(msgs, covers.device)
    a = codec.encode(covers, pl, maps=torch.full((B, pl.map_words), -1, dtype=torch.int64, device=covers.device))
    z = codec.encode(covers, pl, maps=torch.zeros((B, pl.map_words), dtype=torch.int64, device=covers.device))
    assert torch.equal(a.maps, z.maps) and torch.equal(a.stego.view(torch.int16), z.stego.view(torch.int16))


GUARD_CASES = [c for c in CASES if str(c["embedder"]) == "hybrid" and int(c["nbits"]) < 0 and float(c["beta"]) > 0
               and not bool(c["align"])]
GUARD_CASES = list({str(c["image_key"]) + str(c["cover"].shape): c for c in GUARD_CASES}.values())[:6]


@pytest.mark.parametrize("case", GUARD_CASES, ids=[c["name"] for c in GUARD_CASES])
def test_guard_band_ties_fall_back_to_reference_s(case, decide_path):
    """beta set so that beta * H(Y) lands on (and one ulp either side of)
    a prefix sum of the reference's own MI values -- inside the guard band, so the exact
    numpy-order sums must decide, and s must be the reference loop's on its own floats
    (codec.py:580-593 over the golden MI table).  Far from a tie the fast route decides."""
    mis = [float(x) for x in case["mi"]]
    H = float(case["entropy"])
    cover = case["cover"]
    ncheck = 0
    c = 0.0
    for k in range(min(len(mis), 6)):
        c += mis[k]
        if c <= 0.0:
            continue
        b0 = c / H
        for beta in (b0, float(np.nextafter(b0, 0.0)), float(np.nextafter(b0, 2.0))):
            _, enc = _run_case(case, all_mi=False, beta=beta)
            m = enc.records()[0]
            s_ref, cum_ref = _ref_loop(mis, H, beta)
            assert m.status == 0
            assert m.s == s_ref, (k, beta)
            assert m.flags & _lib.FLAG_GUARD_FALLBACK, (k, beta)
            assert not (m.flags & _lib.FLAG_INFO_FAST)
            assert m.cum_info == cum_ref, (k, beta)
            ev = _ref_evaluated(mis, H, beta)
            assert [m.mi[i] for i in range(ev)] == mis[:ev]
            ncheck += 1
    assert ncheck >= 3
    # midway between two prefix sums: far from any tie, decided without the joint sums
    c0, c1 = mis[0], mis[0] + mis[1]
    if c1 - c0 > 1e-6:
        beta = (c0 + c1) / 2 / H
        _, enc = _run_case(case, all_mi=False, beta=beta)
        m = enc.records()[0]
        assert m.flags & _lib.FLAG_INFO_FAST and m.s == _ref_loop(mis, H, beta)[0] == 2


def _mixed_covers(kind, n, h, w, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = kind[i % len(kind)]
        if k == "smooth":     # few values, large counts (a low-entropy slice: small H(Y))
            y, x = np.mgrid[:h, :w]
            out.append((((x // 7 + y // 5) % 9) * 3 + rng.integers(0, 2, (h, w))).astype(np.uint16))
        elif k == "sparse":   # ~200 distinct 16-bit values
            vals = np.sort(rng.choice(65536, 200, replace=False)).astype(np.uint16)
            out.append(vals[rng.integers(0, vals.size, (h, w))])
        else:
            out.append(synth.GENERATORS[k](h, w, seed + i))
    return np.stack(out)


@pytest.mark.parametrize("dtype", ["uint16", "uint8"])
def test_guard_band_random_betas_batch(dtype, decide_path):
    """The guard-banded decision over a mixed batch and a sweep of beta, including betas one
    part in 1e12 from a slice's prefix tie (inside the band: that slice falls back to the exact
    sums while the others of the same launch take the fast route): s equals the reference
    loop's on the oracle's float64 MI values (oracle/ref_cpu.py, pinned to the reference)."""
    kinds = ["ct12", "u16", "smooth", "sparse"] if dtype == "uint16" else ["u8"]
    B, h, w = 12, 96, 128
    covers = _mixed_covers(kinds, B, h, w, 77) if dtype == "uint16" else \
        np.stack([synth.u8(h, w, 70 + i) for i in range(B)])
    nb = 8 * covers.dtype.itemsize
    tabs = []
    for i in range(B):
        mis = [R.mutual_information((covers[i] >> p) & 1, covers[i]) for p in range(nb)]
        tabs.append((mis, R.entropy(covers[i])))
    betas = [0.0, 0.05, 0.2, 0.35, 0.5, 0.65, 0.8, 0.95, 1.0, 1.2]
    for i in (1, 2, 5):   # near-ties of slice i's prefix 2
        c = sum(tabs[i][0][:2])
        if c > 0:
            b0 = c / tabs[i][1]
            betas += [b0 * (1 + 1e-12), b0 * (1 - 1e-12)]
    msgs = [synth.payload(20 + 3 * i, 500 + i) for i in range(B)]
    fallbacks = 0
    for beta in betas:
        codec = Codec(B, h, w, dtype=dtype, beta=beta, block=16)
        enc = codec.encode(torch.from_numpy(covers).cuda(), msgs)
        for i, m in enumerate(enc.records()):
            assert m.s == _ref_loop(tabs[i][0], tabs[i][1], beta)[0], (beta, i)
            assert m.entropy == tabs[i][1]
            fallbacks += bool(m.flags & _lib.FLAG_GUARD_FALLBACK)
    assert fallbacks >= 1        # the near-tie betas reached the exact sums
