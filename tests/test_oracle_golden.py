"""Pin the CPU oracle (oracle/ref_cpu.py) to the reference's own outputs.

Every expected value here was produced by the reference (`src/codec.py`) itself, via
tests/golden/make_golden.py.  The oracle must reproduce all of it bit-for-bit before
it is trusted as the checker for the HIP path.
"""
import numpy as np
import pytest

import golden_io
from oracle import ref_cpu as R

CASES = golden_io.cases()
IDS = [c["name"] for c in CASES]


def _embed(case):
    cover = case["cover"]
    nb = int(case["nbits"])
    gl, loc = R.decompose(cover, beta=float(case["beta"]), nbits=None if nb < 0 else nb)
    bits = str(case["bits"])
    emb = str(case["embedder"])
    sb = int(case["sb"])
    if emb == "hybrid":
        st, maps, used, lens, perm = R.embed_hybrid(loc, bits, search_block_size=sb,
                                                    align_across_planes=bool(case["align"]))
    elif emb == "multi":
        st, maps, used, lens, perm = R.embed_multi_plane(loc, bits)
    else:
        st, maps, used, lens, perm = R.embed_block_adaptive(loc, bits, block_size=sb)
    return gl, loc, st, maps, used, lens, perm


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_oracle_matches_reference(case):
    gl, loc, st, maps, used, lens, perm = _embed(case)
    s = len(loc)
    assert s == int(case["s"])
    assert list(perm) == list(case["perm"])
    assert list(lens) == list(case["sizes"])
    assert used == int(case["total_used"])
    stego = R.merge(gl, st)
    exp = golden_io.stego(case)
    assert stego.dtype == exp.dtype
    np.testing.assert_array_equal(stego, exp)
    np.testing.assert_array_equal(np.stack(maps, 0).astype(np.uint8), golden_io.dense_bitmaps(case))
    flat = np.split(np.stack(maps, 0).reshape(-1), s)
    md = {"s": s, "segments_indices": perm, "segments_lengths": lens}
    assert R.decode_message(R.extract_local_planes(stego, s), flat, md) == golden_io.decoded(case)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_oracle_information_values(case):
    cover = case["cover"]
    assert R.entropy(cover) == float(case["entropy"])
    mi = [R.mutual_information((cover >> i) & 1, cover) for i in range(len(case["mi"]))]
    assert mi == list(case["mi"])


HYBRID_TILING = [c for c in CASES if str(c["embedder"]) == "hybrid" and min(c["sizes"]) >= 0
                 and int(c["nbits"]) < 0]


@pytest.mark.parametrize("case", HYBRID_TILING, ids=[c["name"] for c in HYBRID_TILING])
def test_positional_decode_recovers_payload_and_cover(case):
    """the reference's outputs carry enough to recover payload and cover
    exactly; the positional decoder does it (wrap-free and wrapping windows alike)."""
    stego = golden_io.stego(case)
    maps = golden_io.dense_bitmaps(case)
    s = int(case["s"])
    bits, cover = R.positional_decode(stego, list(maps), s, list(case["perm"]), list(case["sizes"]),
                                      int(case["sb"]), bool(case["align"]))
    npx = stego.size
    payload = str(case["bits"])
    if all(min(max(int(x), 0), npx) == int(x) for x in case["sizes"]):
        assert bits == payload
    np.testing.assert_array_equal(cover, case["cover"])


def test_segment_tables():
    t = golden_io.tables()
    for key in t.files:
        if not key.startswith("seg/") or not key.endswith("/sizes"):
            continue
        _, s, T, _ = key.split("/")
        s, T = int(s), int(T)
        sizes, perm, spans = R.segment_layout(s, T)
        assert sizes == list(t[key]), key
        assert perm == list(t[f"seg/{s}/{T}/perm"]), key
        assert [b - a for a, b in spans] == list(t[f"seg/{s}/{T}/seglens"]), key


def test_entropy_tables():
    t = golden_io.tables()
    names = sorted({k.split("/")[1] for k in t.files if k.startswith("ent/")})
    assert names
    for n in names:
        x = t[f"ent/{n}/x"]
        assert R.entropy(x) == float(t[f"ent/{n}/H"]), n
        mi = [R.mutual_information((x >> i) & 1, x) for i in range(x.dtype.itemsize * 8)]
        assert mi == list(t[f"ent/{n}/mi"]), n


def test_message_to_bits_matches_reference_cases():
    n = 0
    for c in CASES:
        m = golden_io.message(c)
        if m is not None:
            assert R.message_to_bits(m) == str(c["bits"])
            n += 1
    assert n > 10
