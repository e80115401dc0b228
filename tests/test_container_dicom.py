"""STGC container and DICOM I/O: byte-level parity with the reference (CPU) and the
file-level encode/decode pipeline (GPU)."""
import json
import os
import struct

import numpy as np
import pytest

import golden_io
from codec_tcc_amd import container, dicom

Z = np.load(os.path.join(golden_io.GOLDEN, "container.npz"), allow_pickle=False)
NAMES = [str(n) for n in Z["__names__"]]
CASES = {c["name"]: c for c in golden_io.cases()}


@pytest.mark.parametrize("name", NAMES)
def test_container_bytes_match_reference(name, tmp_path):
    c = CASES[name]
    s = int(c["s"])
    h, w = c["cover"].shape
    dense = golden_io.dense_bitmaps(c)
    blob = container.bitmaps_blob(dense)
    codec = str(Z[f"{name}/codec"])
    hdr = container.create_header(codec, s, list(c["sizes"]), list(c["perm"]), len(blob), w, h, 0, False)
    fake = Z[f"{name}/fake_stego"].tobytes()
    path = str(tmp_path / "x.bin")
    size = container.create_binary_file(path, hdr, fake, blob)
    data = open(path, "rb").read()
    assert data == Z[f"{name}/file"].tobytes()
    assert size == int(Z[f"{name}/file_size"])
    md, bm, st = container.parse_bin_file(path)
    ref = json.loads(Z[f"{name}/parsed_json"].tobytes().decode())
    md1 = dict(md)
    md1.pop("version") and ref.pop("version")
    assert md1 == ref
    assert bm == blob and st == fake
    planes = container.split_bitmaps(bm, s)
    np.testing.assert_array_equal(np.stack(planes).reshape(dense.shape), dense)


def test_header_overflow_raises_like_reference():
    assert str(Z["err/big_offset"]) == "error"
    assert str(Z["err/neg_seglen"]) == "error"
    with pytest.raises(struct.error):
        container.create_header("jxl", 1, [1], [0], 1, 4, 4, 70000, False)
    with pytest.raises(struct.error):
        container.create_header("jxl", 1, [-1], [0], 1, 4, 4, 0, False)


def test_container_v2_roundtrip(tmp_path):
    hdr = container.create_header("raw", 3, [5000000, -2, 7], [1, 0, 2], 10, 70000, 3, 123456, True, version=2)
    path = str(tmp_path / "v2.bin")
    container.create_binary_file(path, hdr, b"payload", b"0123456789")
    md, bm, st = container.parse_bin_file(path)
    assert md["version"] == 2 and md["width"] == 70000 and md["start_offset"] == 123456
    assert md["segments_lengths"] == [5000000, -2, 7] and md["segments_indices"] == [1, 0, 2]
    assert md["align_flag"] == 1 and bm == b"0123456789" and st == b"payload"


def test_bad_signature():
    with pytest.raises(ValueError):
        container.parse_bin_bytes(b"XXXX" + b"\x00" * 20)


def _dicom_file(name):
    hz = np.load(os.path.join(golden_io.GOLDEN, "dicom_headers.npz"))
    px = golden_io.images()[name]
    return hz[f"{name}_head"].tobytes() + px.astype(px.dtype.newbyteorder("<")).tobytes() + hz[f"{name}_tail"].tobytes()


@pytest.mark.parametrize("name", ["pe", "torax"])
def test_read_reference_dicoms(name):
    arr, info = dicom.read_dicom(_dicom_file(name))
    exp = golden_io.images()[name]
    assert arr.dtype == exp.dtype and arr.shape == exp.shape
    np.testing.assert_array_equal(arr, exp)
    assert info["transfer_syntax"] in (dicom.EXPLICIT_LE, dicom.IMPLICIT_LE)


@pytest.mark.parametrize("dt", [np.uint8, np.uint16])
def test_dicom_writer_roundtrip(dt, tmp_path):
    img = (np.arange(37 * 41).reshape(37, 41) * 7).astype(dt)
    p = str(tmp_path / "x.dcm")
    dicom.save_dicom(img, p)
    back, info = dicom.read_dicom(p)
    np.testing.assert_array_equal(back, img)
    assert info["bits_allocated"] == 8 * np.dtype(dt).itemsize
    assert info["bits_stored"] == min(int(np.ceil(np.log2(float(img.max()) + 1))), 8 * np.dtype(dt).itemsize)
    with pytest.raises(ValueError):
        dicom.create_dicom_bytes(img.astype(np.int32))
    with pytest.raises(ValueError):
        dicom.create_dicom_bytes(img[None])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pe", "torax"])
def test_file_pipeline_gpu(name, tmp_path):
    """main()-style encode to .bin from the DICOM file, then decode_bin (reference output,
    bit-exact) and the exact decoder (payload + cover)."""
    pytest.importorskip("torch")
    from codec_tcc_amd import pipeline
    from oracle import ref_cpu as R
    src = str(tmp_path / f"{name}.dcm")
    open(src, "wb").write(_dicom_file(name))
    msg = "Mensagem de teste para esteganografia!"
    out = str(tmp_path / "saida.bin")
    info = pipeline.encode_file(src, msg, out, beta=0.4, block=16, codec="raw")
    assert info["version"] == 1
    golden = CASES[f"{name}_b0.4_main"]
    np.testing.assert_array_equal(info["stego"], golden_io.stego(golden))
    message, stego = pipeline.decode_bin(out, output_prefix=str(tmp_path / "dec"))
    assert message == golden_io.decoded(golden)
    np.testing.assert_array_equal(stego, golden_io.stego(golden))
    assert open(str(tmp_path / "dec_mensagem.txt"), encoding="utf-8").read() == message
    np.testing.assert_array_equal(dicom.read_dicom(str(tmp_path / "dec_imagem.dcm"))[0], stego)
    bits, cover = pipeline.decode_bin_exact(out)
    assert bits == R.message_to_bits(msg)
    np.testing.assert_array_equal(cover, golden_io.images()[name])


@pytest.mark.parametrize("dt", [np.uint8, np.uint16])
def test_deflated_dicom_roundtrip(dt):
    """The reference's 'png' codec = a Deflated Explicit VR LE DICOM (codec.py:151-162,
    203-206): the dataset after the file meta is one raw deflate stream.  Byte parity with
    pydicom's writer is unpinned (pydicom is absent); the pixel round trip is exact."""
    import zlib
    img = (np.arange(64 * 48).reshape(64, 48) * 13 % (4096 if dt == np.uint16 else 256)).astype(dt)
    data = dicom.create_dicom_bytes(img, transfer_syntax=dicom.DEFLATED_LE)
    back, info = dicom.read_dicom(data)
    assert info["transfer_syntax"] == dicom.DEFLATED_LE
    np.testing.assert_array_equal(back, img)
    plain = dicom.create_dicom_bytes(img)
    i = plain.index(b"DICM") + 4
    meta_len = 12 + struct.unpack_from("<I", plain, i + 8)[0]
    meta_len_d = 12 + struct.unpack_from("<I", data, i + 8)[0]
    # the body after the (group-length-framed) file meta inflates to the plain dataset
    assert zlib.decompress(data[i + meta_len_d:], -15) == plain[i + meta_len:]
    assert len(data) < len(plain)


def test_container_v2_block_field(tmp_path):
    hdr = container.create_header("raw", 2, [3, 4], [1, 0], 5, 9, 9, 77, False, version=2, search_block_size=8)
    path = str(tmp_path / "b.bin")
    container.create_binary_file(path, hdr, b"px", b"01234")
    md, bm, st = container.parse_bin_file(path)
    assert md["search_block_size"] == 8 and md["start_offset"] == 77 and bm == b"01234" and st == b"px"
    hdr = container.create_header("raw", 2, [3, 4], [1, 0], 5, 9, 9, 77, False, version=2)
    container.create_binary_file(path, hdr, b"px", b"01234")
    assert "search_block_size" not in container.parse_bin_file(path)[0]


def test_pee_container_roundtrip(tmp_path):
    lm = np.random.default_rng(3).random(1237) < 0.1
    blob = container.lm_blob(lm)
    hdr = container.create_pee_header("png", 2, 512, 510, 3, 8192, 1236, 4095, 0, len(blob))
    path = str(tmp_path / "p.bin")
    container.create_binary_file(path, hdr, b"stego-bytes", blob)
    md, bm, st = container.parse_pee_bytes(open(path, "rb").read())
    assert (md["codec"], md["bytes"], md["width"], md["height"]) == ("png", 2, 512, 510)
    assert (md["T"], md["L"], md["end"], md["maxval"], md["status"]) == (3, 8192, 1236, 4095, 0)
    assert st == b"stego-bytes"
    np.testing.assert_array_equal(container.lm_from_blob(bm, md["end"]), lm)
    with pytest.raises(ValueError):
        container.parse_bin_file(path)            # the LSB parser refuses a PEE file
    with pytest.raises(ValueError):
        container.parse_pee_bytes(b"STGC" + struct.pack(">I", 1) + b"\x01")


def test_pee2_container_roundtrip(tmp_path):
    """Scheme 2's header (scheme byte 2, four passes' records and maps) round-trips, and each
    scheme's parser refuses the other's files."""
    rng = np.random.default_rng(4)
    lms = [rng.random(n) < 0.1 for n in (300, 17, 0, 5)]
    blobs = [container.lm_blob(m) if m.size else b"" for m in lms]
    passes = [(120, 299, 1, len(blobs[0])), (40, 16, 0, len(blobs[1])), (0, -1, 0, 0), (9, 4, 0, len(blobs[3]))]
    hdr = container.create_pee2_header("raw", 2, 64, 48, 2, 4095, 169, 0, passes)
    path = str(tmp_path / "p2.bin")
    container.create_binary_file(path, hdr, b"stego-bytes", b"".join(blobs))
    raw = open(path, "rb").read()
    assert container.pee_scheme(raw) == 2
    md, bl, st = container.parse_pee2_bytes(raw)
    assert (md["codec"], md["bytes"], md["width"], md["height"], md["T"], md["maxval"], md["L"], md["status"]) == \
        ("raw", 2, 64, 48, 2, 4095, 169, 0)
    assert st == b"stego-bytes"
    for p, (ps, m) in enumerate(zip(md["passes"], lms)):
        assert (ps["L"], ps["end"], ps["status"]) == passes[p][:3]
        if ps["end"] >= 0:
            np.testing.assert_array_equal(container.lm_from_blob(bl[p], ps["end"]), m[: ps["end"] + 1])
    with pytest.raises(ValueError, match="scheme-2"):
        container.parse_pee_bytes(raw)
    one = container.create_pee_header("raw", 2, 8, 8, 2, 0, -1, 4095, 0, 0)
    container.create_binary_file(path, one, b"x", b"")
    assert container.pee_scheme(open(path, "rb").read()) == 1
    with pytest.raises(ValueError):
        container.parse_pee2_bytes(open(path, "rb").read())
    bad = bytearray(hdr)
    bad[3] = 7
    container.create_binary_file(path, bytes(bad), b"x", b"")
    with pytest.raises(ValueError, match="scheme byte"):
        container.pee_scheme(open(path, "rb").read())


def test_j2k_jls_raise_clearly():
    from codec_tcc_amd import pipeline
    for c in ("j2k", "jls"):
        with pytest.raises(RuntimeError, match="gdcmconv"):
            pipeline._compress(np.zeros((4, 4), np.uint16), c)
        with pytest.raises(RuntimeError, match="gdcmconv"):
            pipeline._decompress(b"", c, 4, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pe", "torax"])
def test_file_pipeline_png_gpu(name, tmp_path):
    """The 'png' (deflated DICOM) stego codec through encode_file -> decode_bin /
    decode_bin_exact: the reference's stego and message bit for bit, exact payload + cover.
    Also version 2 (stored offset and block size, block 8)."""
    pytest.importorskip("torch")
    from codec_tcc_amd import pipeline
    from oracle import ref_cpu as R
    src = str(tmp_path / f"{name}.dcm")
    open(src, "wb").write(_dicom_file(name))
    msg = "Mensagem de teste para esteganografia!"
    out = str(tmp_path / "saida.bin")
    info = pipeline.encode_file(src, msg, out, beta=0.4, block=16, codec="png")
    golden = CASES[f"{name}_b0.4_main"]
    np.testing.assert_array_equal(info["stego"], golden_io.stego(golden))
    message, stego = pipeline.decode_bin(out)
    assert message == golden_io.decoded(golden)
    np.testing.assert_array_equal(stego, golden_io.stego(golden))
    bits, cover = pipeline.decode_bin_exact(out)
    assert bits == R.message_to_bits(msg)
    np.testing.assert_array_equal(cover, golden_io.images()[name])
    out2 = str(tmp_path / "v2.bin")
    img = golden_io.images()[name]
    info2 = pipeline.encode_file(img, msg, out2, beta=0.4, block=8, codec="png", version=2)
    exp = R.encode_slice(img, R.message_to_bits(msg), beta=0.4, sb=8)
    assert info2["start_offset"] == exp["start_offset"]
    np.testing.assert_array_equal(info2["stego"], exp["stego"])
    bits2, cover2 = pipeline.decode_bin_exact(out2)            # block 8 and the offset from the header
    assert bits2 == R.message_to_bits(msg)
    np.testing.assert_array_equal(cover2, img)


@pytest.mark.gpu
@pytest.mark.parametrize("name,codec,T", [("pe", "raw", 2), ("pe", "png", "auto"), ("torax", "png", 2)])
def test_pee_file_pipeline_gpu(name, codec, T, tmp_path):
    """C5 with the north star's algorithm: MED-PEE on the reference's real DICOMs, maxval
    from BitsStored (pe.dcm: 12 bits -> 4095, overflow candidates in the location map),
    written to a version-16 STGC file and recovered exactly from the file alone."""
    pytest.importorskip("torch")
    from codec_tcc_amd import framing, pipeline
    from oracle import pee_cpu as P
    src = str(tmp_path / f"{name}.dcm")
    open(src, "wb").write(_dicom_file(name))
    img = golden_io.images()[name]
    maxval = 4095 if name == "pe" else 255
    payload = "".join(chr(32 + (i * 7) % 95) for i in range(600))
    bits = framing.to_bits(payload)
    out = str(tmp_path / "pee.bin")
    info = pipeline.encode_file_pee(src, payload, out, T=T, codec=codec)
    assert info["maxval"] == maxval and info["status"] == 0
    Texp = P.select_T(img, bits.size, 16, maxval) if T == "auto" else T
    st, side = P.pee_embed(img, bits, Texp, maxval=maxval)
    assert info["T"] == Texp and info["end"] == side["end"]
    np.testing.assert_array_equal(info["stego"], st)
    got, cover = pipeline.decode_bin_pee(out)
    np.testing.assert_array_equal(got, bits)
    np.testing.assert_array_equal(cover, img)
    if name == "pe":
        assert info["lm_count"] > 0 or side["lm"].sum() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,codec,T", [("pe", "raw", 1), ("torax", "png", 2)])
def test_pee2_file_pipeline_gpu(name, codec, T, tmp_path):
    """C5 with scheme 2: the reference's DICOMs, four sublattice passes, a version-16 file with
    scheme byte 2 (every pass's record and map), recovered exactly from the file alone; the
    stego equals the oracle's."""
    pytest.importorskip("torch")
    from codec_tcc_amd import framing, pipeline
    from oracle import pee_cpu as P
    src = str(tmp_path / f"{name}.dcm")
    open(src, "wb").write(_dicom_file(name))
    img = golden_io.images()[name]
    maxval = 4095 if name == "pe" else 255
    payload = "".join(chr(32 + (i * 11) % 95) for i in range(900))
    bits = framing.to_bits(payload)
    out = str(tmp_path / "pee2.bin")
    info = pipeline.encode_file_pee(src, payload, out, T=T, codec=codec, scheme=2)
    st, side = P.pee_embed_multi(img, bits, T, maxval=maxval)
    assert info["scheme"] == 2 and info["status"] == side["status"] and info["L"] == side["L"]
    assert [p["L"] for p in info["passes"]] == [p["L"] for p in side["passes"]]
    np.testing.assert_array_equal(info["stego"], st)
    got, cover = pipeline.decode_bin_pee(out)
    np.testing.assert_array_equal(got, bits[: side["L"]])
    np.testing.assert_array_equal(cover, img)


_FAKE_CJXL = '''import sys
a = sys.argv[1:]
# the reference's command line: cjxl <in.png> <out.jxl> -d 0 -e 3 (codec.py:121)
assert len(a) == 6 and a[2:] == ["-d", "0", "-e", "3"] and a[0].endswith(".png") and a[1].endswith(".jxl"), a
data = open(a[0], "rb").read()
assert data[:8] == b"\\x89PNG\\r\\n\\x1a\\n"
open(a[1], "wb").write(b"FAKEJXL1" + data)
open(__file__ + ".log", "a").write(" ".join(["cjxl"] + a[2:]) + "\\n")
'''
_FAKE_DJXL = '''import sys
a = sys.argv[1:]
# djxl <in.jxl> <out.png> (codec.py:175)
assert len(a) == 2 and a[0].endswith(".jxl") and a[1].endswith(".png"), a
d = open(a[0], "rb").read()
assert d[:8] == b"FAKEJXL1"
open(a[1], "wb").write(d[8:])
open(__file__ + ".log", "a").write("djxl\\n")
'''


@pytest.mark.parametrize("name", ["pe_b0.4_1k", "torax_b0.4_1k"])
def test_jxl_plumbing_with_stand_in_binaries(name, tmp_path, monkeypatch):
    """C5's JPEG-XL leg (pipeline.py _compress/_decompress, codec.py:111-129 / 169-182) run end
    to end with stand-in cjxl/djxl on PATH (the real binaries are absent: .MISSING_LARGE_BLOBS).
    The stand-ins assert the reference's argument vectors and pass the 16-bit PNG through, so
    what is checked is this build's side: the PNG it writes (the reference's
    Image.fromarray(stego.astype(uint16))), the file layout, and the PNG it reads back --
    bit-exact, a uint8 stego coming back as uint16 exactly as in the reference.  decode_bin then
    runs on the .bin with its two GPU calls (extract_local_planes, decode_message) replaced by
    the oracle's, and returns the reference's own decoded message (golden)."""
    import sys
    from codec_tcc_amd import api, pipeline
    from oracle import ref_cpu as R
    pytest.importorskip("PIL")
    bind = tmp_path / "bin"
    bind.mkdir()
    for exe, body in (("cjxl", _FAKE_CJXL), ("djxl", _FAKE_DJXL)):
        p = bind / exe
        p.write_text(f"#!{sys.executable}\n" + body)
        p.chmod(0o755)
    monkeypatch.setenv("PATH", str(bind) + os.pathsep + os.environ.get("PATH", ""))
    case = CASES[name]
    stego = golden_io.stego(case)
    h, w = stego.shape
    data = pipeline._compress(stego, "jxl")
    assert data[:8] == b"FAKEJXL1"
    back = pipeline._decompress(data, "jxl", h, w)
    assert back.dtype == np.uint16 and back.shape == (h, w)
    np.testing.assert_array_equal(back, stego.astype(np.uint16))
    # the whole file: header + jxl stego + zlib bitmaps -> decode_bin (GPU calls -> oracle)
    s = int(case["s"])
    blob = container.bitmaps_blob(golden_io.dense_bitmaps(case).astype(np.uint8))
    hdr = container.create_header("jxl", s, [int(x) for x in case["sizes"]], [int(x) for x in case["perm"]],
                                  len(blob), w, h, 0, False)
    out = str(tmp_path / "saida.bin")
    container.create_binary_file(out, hdr, data, blob)
    monkeypatch.setattr(api, "extract_local_planes", R.extract_local_planes)
    monkeypatch.setattr(api, "decode_message", R.decode_message)
    message, st = pipeline.decode_bin(out)
    np.testing.assert_array_equal(st, stego.astype(np.uint16))
    assert message == golden_io.decoded(case)
    log = (bind / "cjxl.log").read_text().split("\n") + (bind / "djxl.log").read_text().split("\n")
    assert "cjxl -d 0 -e 3" in log and log.count("djxl") == 2
