"""CPU-only checks: host framing logic vs the reference's tables, the C-ABI library's
exports, struct layouts, numpy semantics the device emulates, and failure without GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import golden_io
from codec_tcc_amd import _lib, framing

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_segment_plan_matches_reference_tables():
    t = golden_io.tables()
    n = 0
    for key in t.files:
        if key.startswith("seg/") and key.endswith("/sizes"):
            _, s, T, _ = key.split("/")
            sizes, perm, spans = framing.segment_plan(int(s), int(T))
            assert list(sizes) == list(t[key])
            assert list(perm) == list(t[f"seg/{s}/{T}/perm"])
            assert [b - a for a, b in spans] == list(t[f"seg/{s}/{T}/seglens"])
            n += 1
    assert n == 16 * 20


def test_message_to_bits_and_packing_roundtrip():
    for c in golden_io.cases():
        m = golden_io.message(c)
        if m is None:
            continue
        assert framing.message_to_bits(m) == str(c["bits"])
        bits = framing.to_bits(m)
        words, lens = framing.pack_bits([bits])
        back = framing.unpack_bits(words[0], lens[0])
        assert framing.bits_to_str(back) == str(c["bits"])


def test_distribute_message_segments_dropin():
    segs, sizes, perm = framing.distribute_message_segments([0] * 4, "1011" * 10)
    assert sizes == [22, 12, 5, 1] and perm == [2, 1, 3, 0]
    assert "".join(segs) == "1011" * 10


def test_layout_table_rows():
    table, cls, n = framing.layout_table([320, 320, 8192])
    assert n == 2 and list(cls) == [0, 0, 1]
    rows = (_lib.Layout * (16 * n)).from_buffer_copy(table)
    r = rows[16 * 1 + 4]   # T=8192, s=5
    sizes, perm, spans = framing.segment_plan(5, 8192)
    assert [r.perm[j] for j in range(5)] == list(perm)
    assert [r.sizes[p] for p in range(5)] == list(sizes)
    assert sum(r.len[p] for p in range(5)) == 8192


def test_global_random_state_untouched():
    import random
    random.seed(123)
    a = random.random()
    random.seed(123)
    framing.plane_order.cache_clear()
    framing.plane_order(7)
    assert random.random() == a


def test_struct_layout_matches_header():
    """ctypes mirrors of codec_tcc.h: sizes must match the C compiler's view."""
    hdr = os.path.join(REPO, "include", "codec_tcc.h")
    src = f'#include "{hdr}"\n#include <stdio.h>\n#include <stddef.h>\nint main(){{printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(codec_params), sizeof(codec_layout), sizeof(codec_slice_meta), offsetof(codec_slice_meta, entropy), offsetof(codec_slice_meta, mi), sizeof(codec_pee_params), sizeof(codec_pee_meta), offsetof(codec_slice_meta, span_lo), offsetof(codec_pee_meta, lm_count));return 0;}}\n'
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        cpath = os.path.join(d, "t.c")
        open(cpath, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", cpath, "-o", exe])
        out = subprocess.check_output([exe]).decode().split()
    sizes = list(map(int, out))
    assert sizes[0] == C.sizeof(_lib.Params)
    assert sizes[1] == C.sizeof(_lib.Layout)
    assert sizes[2] == C.sizeof(_lib.SliceMeta)
    assert sizes[3] == _lib.SliceMeta.entropy.offset
    assert sizes[4] == _lib.SliceMeta.mi.offset
    assert sizes[5] == C.sizeof(_lib.PeeParams)
    assert sizes[6] == C.sizeof(_lib.PeeMeta) == _lib.PEE_META_BYTES
    assert sizes[7] == _lib.SliceMeta.span_lo.offset
    assert sizes[8] == _lib.PeeMeta.lm_count.offset


def test_library_digest_ties_binary_to_sources(monkeypatch, tmp_path):
    """the in-tree library carries the digest of the sources it was built
    from; the loader refuses it when the tree's digest differs (a stale or copied-in binary),
    and a library without any digest is refused too."""
    from codec_tcc_amd import build
    if build.needs_build():
        build.build()
    assert build.library_digest() == build.source_digest()
    monkeypatch.setattr(_lib, "_lib", None)                 # force a fresh load
    monkeypatch.setattr(build, "source_digest", lambda *a, **k: "0" * 64)
    with pytest.raises(RuntimeError, match="not built from these sources"):
        _lib.load()
    monkeypatch.undo()
    fake = tmp_path / "libcodec_hip.so"
    fake.write_bytes(b"\x7fELF no digest here")
    assert build.library_digest(str(fake)) is None
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "_DEFAULT_PATH", str(fake))
    with pytest.raises(RuntimeError, match="not built from these sources"):
        _lib.load(str(fake))
    monkeypatch.undo()
    assert _lib.load().codec_build_digest().decode() == build.source_digest()


@pytest.mark.filterwarnings("ignore:.*non-default flags:RuntimeWarning")   # this test fakes another environment
def test_library_digest_uses_the_flags_it_was_built_with(monkeypatch):
    """the build flags travel inside the library, so a process whose environment
    would build with other flags (CODEC_OFFLOAD_ARCH / CODEC_BUILD_DEFS) still loads it; a
    tree without the sources fails with a clear message, not an OSError."""
    from codec_tcc_amd import build
    if build.needs_build():
        build.build()
    assert build.library_flags() == build.FLAGS
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(build, "FLAGS", build.FLAGS + ["-DSOME_OTHER_BUILD"])
    assert _lib.load() is not None
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(build, "SRCS", build.SRCS + [os.path.join(REPO, "codec_tcc_amd", "csrc", "absent.hip")])
    with pytest.raises(RuntimeError, match="absent"):
        _lib.load()
    monkeypatch.undo()
    assert _lib.load() is not None


def test_library_exports_every_header_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        from codec_tcc_amd import build
        build.build()
    hdr = open(os.path.join(REPO, "include", "codec_tcc.h")).read()
    declared = set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(codec_\w+)\s*\(", hdr, re.M))
    assert declared == set(_lib.EXPORTS)
    lib = _lib.load()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.codec_abi_version() == 1
    P = _lib.Params(B=2, H=64, W=64, in_bytes=2, out_bytes=2, nbits=16, block=16, align=0, mode=0,
                    fixed_s=0, fixed_offset=-1, all_mi=0, payload_words=1, map_words=1, n_classes=1, beta=0.4)
    ws = lib.codec_workspace_bytes(C.byref(P))
    assert ws >= 2 * 65536 * 4
    P.nbits = 17
    assert lib.codec_workspace_bytes(C.byref(P)) == 0
    assert lib.codec_plan(C.byref(P), None, None, None, 0, None, None, None, None, 0, None) < 0
    assert b"nbits" in lib.codec_last_error()


def test_product_path_has_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import codec_tcc_amd as ct
    with pytest.raises(RuntimeError, match="no GPU"):
        ct.encode(np.zeros((16, 16), np.uint16), ["x"])


def test_product_never_imports_oracle():
    pkg = os.path.join(REPO, "codec_tcc_amd")
    for root, _dirs, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(root, f)).read()
                assert "oracle" not in re.sub(r"#.*", "", txt).replace("oracle/", ""), f


# ---- numpy semantics the device emulates (np.sum buffering + pairwise, np.var)
def _pw(a, i0, n):
    if n < 8:
        r = -0.0
        for i in range(n):
            r += a[i0 + i]
        return r
    if n <= 128:
        r = [a[i0 + j] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[i0 + i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i0 + i]
            i += 1
        return res
    n2 = (n >> 1) & ~7
    return _pw(a, i0, n2) + _pw(a, i0 + n2, n - n2)


def _np_sum_emul(a):
    res = -0.0
    for s in range(0, len(a), 8192):
        res += _pw(a, s, min(8192, len(a) - s))
    return res


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 127, 128, 129, 255, 1000, 8191, 8192, 8193, 20000, 65536, 65537])
def test_numpy_sum_is_buffered_pairwise(n):
    rng = np.random.default_rng(n)
    a = rng.standard_normal(n) * 1e3 - 5
    assert np.sum(a) == _np_sum_emul(list(map(float, a)))


def test_numpy_log2_is_elementwise():
    """The device uses a per-value log2 table; numpy's vectorised log2 must not depend on
    the element's position in the array."""
    x = np.random.default_rng(0).random(10007)
    full = np.log2(x)
    for k in (1, 2, 3, 7, 8, 9, 15, 16, 17):
        for i in range(0, 300):
            assert np.log2(x[i:i + k])[0] == full[i]


def test_loader_refuses_diagnostic_builds(tmp_path, monkeypatch):
    """a diagnostic build (phase stamps, a scan that returns before deciding) carries
    a digest that matches its own flags; the loader still refuses it at the in-tree path unless
    CODEC_ALLOW_DIAG_LIB=1."""
    from codec_tcc_amd import build
    monkeypatch.setattr(build, "library_flags", lambda path=None: build.FLAGS + ["-DDECIDE_TS", "-DDECIDE_TS_SCAN_ONLY"])
    monkeypatch.delenv("CODEC_ALLOW_DIAG_LIB", raising=False)
    with pytest.raises(RuntimeError, match="diagnostic build"):
        _lib._check_digest(_lib.LIB_PATH)
