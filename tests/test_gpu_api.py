"""The drop-in functions (codec_tcc_amd.api, reference names) vs the reference's golden
outputs and the oracle.  GPU only: each call runs the HIP kernels through the C ABI."""
import numpy as np
import pytest

import golden_io
from codec_tcc_amd import api
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
pytest.importorskip("torch")

ALL = golden_io.cases()
PICK = [c for c in ALL if c["name"] in (
    "pe_b0.4_1k", "torax_b0.8_main", "pe_sb8_align", "pe_nbits12", "ct12_37x53", "u8_5x5", "u16_8x8_wrap",
    "ct12_64_sb5", "ct12_64_T2", "u16_1x300", "const_u16", "u16_64_beta0.999", "pe_multi", "u16_8x8_wrap_multi")]


def _bits(case):
    return str(case["bits"])


@pytest.mark.parametrize("case", PICK, ids=[c["name"] for c in PICK])
def test_dropin_pipeline(case):
    cover = case["cover"]
    nb = int(case["nbits"])
    nbits = None if nb < 0 else nb
    gl, loc = api.adaptive_modalities_decomposition(cover, beta=float(case["beta"]), nbits=nbits)
    egl, eloc = R.decompose(cover, beta=float(case["beta"]), nbits=nbits)
    assert len(loc) == int(case["s"]) == len(eloc)
    for a, b in zip(gl + loc, egl + eloc):
        assert a.dtype == b.dtype
        np.testing.assert_array_equal(a, b)
    if str(case["embedder"]) == "hybrid":
        st, maps, used, lens, perm = api.lsb_embed_block_then_multiplane(
            loc, _bits(case), search_block_size=int(case["sb"]), align_across_planes=bool(case["align"]))
    else:
        st, maps, used, lens, perm = api.lsb_embed_multi_plane(loc, _bits(case))
    assert used == int(case["total_used"])
    assert lens == list(case["sizes"]) and perm == list(case["perm"])
    np.testing.assert_array_equal(np.stack(maps, 0), golden_io.dense_bitmaps(case))
    stego = api.merge_modalities(gl, st)
    np.testing.assert_array_equal(stego, golden_io.stego(case))
    s = len(loc)
    planes = api.extract_local_planes(stego, s)
    for a, b in zip(planes, R.extract_local_planes(stego, s)):
        np.testing.assert_array_equal(a, b)
    flat = np.split(np.stack(maps, 0).reshape(-1), s)
    md = {"s": s, "segments_indices": perm, "segments_lengths": lens}
    assert api.decode_message(planes, flat, md) == golden_io.decoded(case)


TILING = [c for c in PICK if str(c["embedder"]) == "hybrid" and min(c["sizes"]) >= 0
          and int(c["nbits"]) < 0 and max(c["sizes"]) <= c["cover"].size]


@pytest.mark.parametrize("case", TILING, ids=[c["name"] for c in TILING])
def test_decode_positional(case):
    stego = golden_io.stego(case)
    maps = golden_io.dense_bitmaps(case)
    s = int(case["s"])
    md = {"s": s, "segments_indices": list(case["perm"]), "segments_lengths": list(case["sizes"])}
    bits, cover = api.decode_positional(stego, list(maps), md, search_block_size=int(case["sb"]),
                                        align_across_planes=bool(case["align"]))
    if sum(case["sizes"]) <= case["cover"].size:
        assert bits == _bits(case)
    np.testing.assert_array_equal(cover, case["cover"])


def test_entropy_and_mi_tables():
    t = golden_io.tables()
    names = sorted({k.split("/")[1] for k in t.files if k.startswith("ent/")})
    for n in names:
        x = t[f"ent/{n}/x"]
        assert api.calculate_entropy(x) == float(t[f"ent/{n}/H"]), n
        mi = t[f"ent/{n}/mi"]
        for i in range(x.dtype.itemsize * 8):
            assert api.calculate_mutual_information((x >> i) & 1, x) == float(mi[i]), (n, i)


def test_errors_like_reference():
    with pytest.raises(ValueError):
        api.adaptive_modalities_decomposition(np.zeros((4, 4), np.float32))
    with pytest.raises(ValueError):
        api.lsb_embed_block_then_multiplane([np.full((4, 4), 2, np.uint16)], "1")


ADAPTIVE = [c for c in ALL if str(c["embedder"]) == "adaptive"]


@pytest.mark.parametrize("case", ADAPTIVE, ids=[c["name"] for c in ADAPTIVE])
def test_block_adaptive_matches_reference(case):
    """lsb_embed_block_adaptive (codec.py:320-410) against the reference's own outputs,
    ravel-copy quirk included (writes only in one-row or full-width blocks)."""
    cover = case["cover"]
    nb = int(case["nbits"])
    gl, loc = api.adaptive_modalities_decomposition(cover, beta=float(case["beta"]),
                                                    nbits=None if nb < 0 else nb)
    st, maps, used, lens, perm = api.lsb_embed_block_adaptive(loc, _bits(case), block_size=int(case["sb"]))
    assert used == int(case["total_used"])
    assert lens == list(case["sizes"]) and perm == list(case["perm"])
    np.testing.assert_array_equal(np.stack(maps, 0), golden_io.dense_bitmaps(case))
    np.testing.assert_array_equal(api.merge_modalities(gl, st), golden_io.stego(case))


def _rand_planes(rng, s, h, w, p_one, dtype):
    return [(rng.random((h, w)) < p_one).astype(dtype) for _ in range(s)]


@pytest.mark.parametrize("h,w,bs,s,nbits,p_one,dtype", [
    (64, 64, 8, 3, 3000, 0.5, np.uint8),       # interior blocks never written (2-D views)
    (65, 40, 8, 2, 900, 0.3, np.uint16),       # bottom block row one pixel high: written
    (200, 6, 8, 4, 1000, 0.5, np.uint8),       # w <= block: every block full-width
    (1, 700, 16, 2, 500, 0.5, np.uint16),      # one row
    (33, 33, 1, 2, 2000, 0.5, np.uint8),       # 1x1 blocks: every block contiguous
    (48, 48, 4, 3, 50000, 0.5, np.uint8),      # payload longer than every plane
    (40, 40, 8, 2, 600, 0.0, np.uint8),        # all-zero planes: ties everywhere (stable order)
    (37, 91, 5, 5, 4000, 0.07, np.uint16),
    (20, 20, 8, 1, 0, 0.5, np.uint8),          # empty message
])
def test_block_adaptive_matches_oracle(h, w, bs, s, nbits, p_one, dtype):
    rng = np.random.default_rng(h * 1000 + w + bs)
    loc = _rand_planes(rng, s, h, w, p_one, dtype)
    bits = "".join("1" if b else "0" for b in rng.integers(0, 2, nbits))
    got = api.lsb_embed_block_adaptive(loc, bits, block_size=bs)
    exp = R.embed_block_adaptive(loc, bits, block_size=bs)
    assert got[2:] == exp[2:]
    for a, b in zip(got[0], exp[0]):
        assert a.dtype == b.dtype
        np.testing.assert_array_equal(a, b)
    for a, b in zip(got[1], exp[1]):
        np.testing.assert_array_equal(a, b)


def test_block_adaptive_rejects_non_binary_planes():
    with pytest.raises(ValueError):
        api.lsb_embed_block_adaptive([np.full((4, 4), 2, np.uint8)], "1")
