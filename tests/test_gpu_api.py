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
