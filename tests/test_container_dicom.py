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
