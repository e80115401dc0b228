#!/usr/bin/env python3
"""Generate the golden vectors that pin `oracle/ref_cpu.py` to the reference.

Run in the BUILD container only (it reads `/root/reference`, which does not exist on
the GPU box):

    python tests/golden/make_golden.py

How the reference is run: `/root/reference/src/codec.py` imports pydicom/pylibjpeg at
module top (codec.py:4,10-16) but none of the hot-path functions use them, so stub
modules are registered in `sys.modules` before loading it.  `sys.dont_write_bytecode`
keeps the read-only reference tree untouched.  Only *data* (inputs and the
reference's outputs) is written here; no reference source is copied.

Outputs (all under tests/golden/):
  images.npz   pixel arrays of images/pe.dcm (uint16, 12-bit) and images/torax.dcm
               (uint8), parsed raw from the DICOM PixelData offsets
  cases.npz    embed/decode cases: inputs + s, perm, sizes, total_used, stego^cover,
               packed dense bitmaps, decode_message() output, entropy, per-plane MI
  tables.npz   distribute_message_segments() sizes/perm for s=1..16 x many T;
               calculate_entropy / calculate_mutual_information on random arrays
  kat2048.json sha256 digests of full-size 2048x2048 encodes
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from codec_tcc_amd import synth  # noqa: E402


def load_reference():
    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m
    root = stub("pydicom")
    stub("pydicom.dataset", FileDataset=object, FileMetaDataset=object)
    stub("pydicom.uid", ExplicitVRLittleEndian=None, generate_uid=lambda: "0",
         JPEGLSLossless=None, JPEG2000Lossless=None,
         DeflatedExplicitVRLittleEndian=None, PYDICOM_IMPLEMENTATION_UID="0")
    stub("pydicom.encaps", encapsulate=None)
    root.config = stub("pydicom.config", image_handlers=[])
    stub("pydicom.pixel_data_handlers", pylibjpeg_handler=None)
    spec = importlib.util.spec_from_file_location("ref_codec", os.path.join(REF, "src", "codec.py"))
    mod = importlib.util.module_from_spec(spec)
    devnull = open(os.devnull, "w")
    old = sys.stdout
    sys.stdout = devnull
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.stdout = old
    return mod


class Quiet:
    def __enter__(self):
        self.old = sys.stdout
        sys.stdout = open(os.devnull, "w")

    def __exit__(self, *a):
        sys.stdout.close()
        sys.stdout = self.old


def dicom_pixels():
    pe = open(os.path.join(REF, "images", "pe.dcm"), "rb").read()
    tx = open(os.path.join(REF, "images", "torax.dcm"), "rb").read()
    pe_px = np.frombuffer(pe[7010:7010 + 524288], dtype="<u2").reshape(512, 512).copy()
    tx_px = np.frombuffer(tx[888:888 + 262144], dtype=np.uint8).reshape(512, 512).copy()
    return pe_px, tx_px


MAIN_MSG = "Mensagem de teste para esteganografia!"   # codec.py:863


def run_case(ref, img, *, beta, sb, align, bits, embedder, nbits=None):
    with Quiet():
        gl, loc = ref.adaptive_modalities_decomposition(img, beta=beta, nbits=nbits)
        if embedder == "hybrid":
            st, maps, used, lens, perm = ref.lsb_embed_block_then_multiplane(
                loc, bits, search_block_size=sb, align_across_planes=align)
        elif embedder == "multi":
            st, maps, used, lens, perm = ref.lsb_embed_multi_plane(loc, bits)
        elif embedder == "adaptive":
            st, maps, used, lens, perm = ref.lsb_embed_block_adaptive(loc, bits, block_size=sb)
        else:
            raise ValueError(embedder)
        stego = ref.merge_modalities(gl, st)
        s = len(loc)
        # decode exactly as decode_bin does (codec.py:820-828): 1-D bitmaps via np.split
        flat = np.split(np.stack(maps, axis=0).reshape(-1), s)
        md = {"s": s, "segments_indices": perm, "segments_lengths": lens}
        dec = ref.decode_message(ref.extract_local_planes(stego, s), flat, md)
        ent = ref.calculate_entropy(img)
        nb = img.dtype.itemsize * 8 if nbits is None else nbits
        mis = [ref.calculate_mutual_information((img >> i) & 1, img) for i in range(nb)]
    out = {
        "s": np.int64(s), "perm": np.asarray(perm, np.int64), "sizes": np.asarray(lens, np.int64),
        "total_used": np.int64(used),
        "stego_dtype": np.array(str(stego.dtype)),
        "bitmaps_packed": np.packbits(np.stack(maps, axis=0).astype(np.uint8).reshape(-1)),
        "decoded_utf8": np.frombuffer(dec.encode("utf-8"), np.uint8), "entropy": np.float64(ent), "mi": np.asarray(mis, np.float64),
    }
    if stego.dtype == img.dtype:
        out["stego_xor"] = stego ^ img
    else:
        out["stego"] = stego
    return out


def main():
    ref = load_reference()
    pe, tx = dicom_pixels()
    np.savez_compressed(os.path.join(HERE, "images.npz"), pe=pe, torax=tx)
    msg1k = synth.payload(1024, 7)

    cases = []   # (name, image-key or array, params)

    def add(name, img, **kw):
        cases.append((name, img, kw))

    # --- real slices (C1 / C5): both images, beta 0.4/0.8, short and 1 KB payloads
    for iname, img in (("pe", pe), ("torax", tx)):
        for beta in (0.4, 0.8):
            for mname, msg in (("main", MAIN_MSG), ("1k", msg1k)):
                add(f"{iname}_b{beta}_{mname}", iname, beta=beta, sb=16, align=False,
                    msg=msg, embedder="hybrid")
    add("pe_sb8_align", "pe", beta=0.4, sb=8, align=True, msg=MAIN_MSG, embedder="hybrid")
    add("pe_nbits12", "pe", beta=0.4, sb=16, align=False, msg=MAIN_MSG, embedder="hybrid", nbits=12)
    add("torax_nbits6", "torax", beta=0.4, sb=16, align=False, msg=MAIN_MSG, embedder="hybrid", nbits=6)
    add("pe_multi", "pe", beta=0.4, sb=16, align=False, msg=msg1k, embedder="multi")
    add("torax_adaptive", "torax", beta=0.4, sb=8, align=False, msg=msg1k, embedder="adaptive")

    # --- synthetic slices: dtypes, odd shapes (partial blocks), block sizes, payload edges
    syn = []
    for seed in range(3):
        syn.append((f"ct12_64_s{seed}", synth.ct12(64, 64, seed), dict(beta=0.4, sb=16, msg=synth.payload(40, seed))))
    syn += [
        ("u16_64", synth.u16(64, 64, 5), dict(beta=0.4, sb=16, msg=synth.payload(40, 1))),
        ("u8_48", synth.u8(48, 48, 6), dict(beta=0.4, sb=16, msg=synth.payload(30, 2))),
        ("ct12_37x53", synth.ct12(37, 53, 3), dict(beta=0.4, sb=16, msg=synth.payload(25, 3))),
        ("u8_100x80", synth.u8(100, 80, 4), dict(beta=0.5, sb=16, msg=synth.payload(60, 4))),
        ("ct12_17x17", synth.ct12(17, 17, 5), dict(beta=0.4, sb=16, msg=synth.payload(8, 5))),
        ("u16_1x300", synth.u16(1, 300, 6), dict(beta=0.4, sb=16, msg=synth.payload(10, 6))),
        ("u16_300x1", synth.u16(300, 1, 7), dict(beta=0.4, sb=16, msg=synth.payload(10, 7))),
        ("u8_5x5", synth.u8(5, 5, 8), dict(beta=0.4, sb=16, msg="ab")),
        ("ct12_64_sb5", synth.ct12(64, 64, 9), dict(beta=0.4, sb=5, msg=synth.payload(40, 9))),
        ("ct12_37x53_sb3", synth.ct12(37, 53, 10), dict(beta=0.4, sb=3, msg=synth.payload(40, 10))),
        ("ct12_64_sb7_align", synth.ct12(64, 64, 11), dict(beta=0.4, sb=7, msg=synth.payload(40, 11), align=True)),
        ("ct12_96_sb32", synth.ct12(96, 96, 12), dict(beta=0.4, sb=32, msg=synth.payload(40, 12))),
        ("u16_64_sb8", synth.u16(64, 64, 13), dict(beta=0.4, sb=8, msg=synth.payload(40, 13))),
        ("u16_8x8_wrap", synth.u16(8, 8, 14), dict(beta=0.4, sb=16, bits="1011" * 50)),
        ("u16_8x8_wrap_align", synth.u16(8, 8, 15), dict(beta=0.4, sb=4, bits="0110" * 40, align=True)),
        ("ct12_64_empty", synth.ct12(64, 64, 16), dict(beta=0.4, sb=16, bits="")),
        ("ct12_64_T1", synth.ct12(64, 64, 17), dict(beta=0.4, sb=16, bits="1")),
        ("ct12_64_T2", synth.ct12(64, 64, 18), dict(beta=0.4, sb=16, bits="10")),
        ("u16_64_T3", synth.u16(64, 64, 19), dict(beta=0.4, sb=16, bits="110")),
        ("ct12_64_unicode", synth.ct12(64, 64, 20), dict(beta=0.4, sb=16, msg="€ção é ok")),
        ("const_u16", np.full((32, 32), 7, np.uint16), dict(beta=0.4, sb=16, msg="hi")),
        ("ct12_64_beta0", synth.ct12(64, 64, 21), dict(beta=0.0, sb=16, msg="x")),
        ("ct12_64_beta1", synth.ct12(64, 64, 22), dict(beta=1.0, sb=16, msg=synth.payload(20, 22))),
        ("ct12_64_beta1.5", synth.ct12(64, 64, 23), dict(beta=1.5, sb=16, msg=synth.payload(20, 23))),
        ("u16_64_beta0.999", synth.u16(64, 64, 24), dict(beta=0.999, sb=16, msg=synth.payload(20, 24))),
        ("twolevel_u16", (np.arange(64 * 64).reshape(64, 64) % 2 * 1000).astype(np.uint16), dict(beta=0.4, sb=16, msg="zz")),
    ]
    syn_arrays = {}
    for name, arr, kw in syn:
        syn_arrays[name] = arr
        kw = dict(kw)
        kw.setdefault("align", False)
        add(name, name, embedder="hybrid", **kw)
    # the other two embedders on a few synthetic slices
    for name in ("ct12_64_s0", "u16_64", "ct12_37x53", "u8_5x5", "u16_8x8_wrap", "ct12_64_T2"):
        kw = dict(next(k for (n, _a, k) in syn if n == name))
        kw.setdefault("align", False)
        add(name + "_multi", name, embedder="multi", **kw)
    for name, bs in (("ct12_64_s1", 8), ("ct12_37x53", 8), ("u16_1x300", 8), ("u16_300x1", 8),
                     ("u8_5x5", 8), ("ct12_17x17", 4), ("u8_100x80", 16)):
        kw = dict(next(k for (n, _a, k) in syn if n == name))
        kw.setdefault("align", False)
        kw["sb"] = bs
        add(name + f"_adaptive{bs}", name, embedder="adaptive", **kw)

    images = {"pe": pe, "torax": tx}
    images.update(syn_arrays)
    out = {}
    names = []
    for name, key, kw in cases:
        img = images[key]
        bits = kw["bits"] if "bits" in kw else ref.message_to_bits(kw["msg"])
        res = run_case(ref, img, beta=kw["beta"], sb=kw["sb"], align=kw.get("align", False),
                       bits=bits, embedder=kw["embedder"], nbits=kw.get("nbits"))
        names.append(name)
        out[f"{name}/image_key"] = np.array(key)
        if key not in ("pe", "torax"):
            out[f"{name}/image"] = img
        out[f"{name}/beta"] = np.float64(kw["beta"])
        out[f"{name}/sb"] = np.int64(kw["sb"])
        out[f"{name}/align"] = np.bool_(kw.get("align", False))
        out[f"{name}/embedder"] = np.array(kw["embedder"])
        out[f"{name}/nbits"] = np.int64(-1 if kw.get("nbits") is None else kw["nbits"])
        out[f"{name}/bits"] = np.array(bits)
        if "msg" in kw:
            out[f"{name}/msg_utf8"] = np.frombuffer(kw["msg"].encode("utf-8"), np.uint8)
        for k, v in res.items():
            out[f"{name}/{k}"] = v
        print(f"{name:28s} s={int(res['s'])} perm={list(res['perm'])} sizes={list(res['sizes'])} used={int(res['total_used'])}")
    out["__names__"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "cases.npz"), **out)

    # --- tables: segment distribution + entropy / MI
    tab = {}
    Ts = [0, 1, 2, 3, 5, 7, 8, 9, 15, 16, 17, 31, 64, 100, 303, 1000, 8192, 8193, 65536, 100003]
    for s in range(1, 17):
        for T in Ts:
            segs, sizes, perm = ref.distribute_message_segments([None] * s, "1" * T)
            tab[f"seg/{s}/{T}/sizes"] = np.asarray(sizes, np.int64)
            tab[f"seg/{s}/{T}/perm"] = np.asarray(perm, np.int64)
            tab[f"seg/{s}/{T}/seglens"] = np.asarray([len(x) for x in segs], np.int64)
    rng = np.random.default_rng(1234)
    ent_arrays = {
        "u8_uniform": rng.integers(0, 256, 5000).astype(np.uint8),
        "u16_uniform": rng.integers(0, 65536, 70000).astype(np.uint16),
        "u16_geom": np.minimum(rng.geometric(0.01, 100000), 65535).astype(np.uint16),
        "u16_12bit": synth.ct12(128, 128, 99),
        "u8_few": rng.integers(0, 3, 777).astype(np.uint8),
        "u16_single": np.full(100, 9, np.uint16),
        "u16_two": np.array([0, 65535] * 50, np.uint16),
        "u16_wide200k": rng.integers(0, 60000, 200000).astype(np.uint16),
    }
    with Quiet():
        for name, arr in ent_arrays.items():
            tab[f"ent/{name}/x"] = arr
            tab[f"ent/{name}/H"] = np.float64(ref.calculate_entropy(arr))
            nb = arr.dtype.itemsize * 8
            tab[f"ent/{name}/mi"] = np.asarray(
                [ref.calculate_mutual_information((arr >> i) & 1, arr) for i in range(nb)], np.float64)
    np.savez_compressed(os.path.join(HERE, "tables.npz"), **tab)

    # --- full-size (2048^2) known answers, stored as digests
    kat = []
    for kind, seed, beta in (("ct12", 0, 0.4), ("u16", 1, 0.4), ("ct12", 2, 0.8)):
        img = synth.GENERATORS[kind](2048, 2048, seed)
        msg = synth.payload(1024, 7 + seed)
        with Quiet():
            gl, loc = ref.adaptive_modalities_decomposition(img, beta=beta)
            st, maps, used, lens, perm = ref.lsb_embed_block_then_multiplane(
                loc, ref.message_to_bits(msg), search_block_size=16)
            stego = ref.merge_modalities(gl, st)
            s = len(loc)
            md = {"s": s, "segments_indices": perm, "segments_lengths": lens}
            flat = np.split(np.stack(maps, axis=0).reshape(-1), s)
            dec = ref.decode_message(ref.extract_local_planes(stego, s), flat, md)
        kat.append({
            "kind": kind, "seed": seed, "beta": beta, "h": 2048, "w": 2048, "payload_seed": 7 + seed,
            "payload_chars": 1024, "s": s, "perm": list(map(int, perm)), "sizes": list(map(int, lens)),
            "total_used": int(used),
            "cover_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
            "stego_sha256": hashlib.sha256(stego.tobytes()).hexdigest(),
            "bitmaps_sha256": hashlib.sha256(np.stack(maps, 0).astype(np.uint8).tobytes()).hexdigest(),
            "decoded_sha256": hashlib.sha256(dec.encode("utf-8")).hexdigest(),
            "decoded_len": len(dec),
        })
        print("kat", kind, seed, "s", s, perm, lens)
    with open(os.path.join(HERE, "kat2048.json"), "w") as f:
        json.dump(kat, f, indent=1)

    # --- container (.bin "STGC", codec.py:601-750) bytes made by the reference itself
    import tempfile
    import zlib
    cont = {}
    with tempfile.TemporaryDirectory() as d:
        k = 0
        for name, codec, fake in (("pe_b0.4_main", "jxl", b"<jxl bytes>"), ("torax_b0.4_1k", "png", b"\x00\x01" * 50),
                                  ("ct12_37x53", "j2k", b""), ("u8_5x5", "weird", b"xyz")):
            res = out  # cases already computed above
            s = int(res[f"{name}/s"])
            perm = [int(x) for x in res[f"{name}/perm"]]
            sizes = [int(x) for x in res[f"{name}/sizes"]]
            key = str(res[f"{name}/image_key"])
            img = images[key]
            h, w = img.shape
            bm = np.unpackbits(res[f"{name}/bitmaps_packed"])[: s * h * w].astype(np.uint8)
            blob = zlib.compress(bm.tobytes())
            with Quiet():
                hdr = ref.create_header(codec=codec, s=s, segments_lengths=sizes, segments_indices=perm,
                                        bitmaps_blob_size=len(blob), width=w, height=h, start_offset=0,
                                        align_across_planes=False)
                path = os.path.join(d, f"c{k}.bin")
                size = ref.create_binary_file(path, hdr, fake, blob)
                md, bmd, stg = ref.parse_bin_file(path)
            data = open(path, "rb").read()
            cont[f"{name}/codec"] = np.array(codec)
            cont[f"{name}/file"] = np.frombuffer(data, np.uint8)
            cont[f"{name}/fake_stego"] = np.frombuffer(fake, np.uint8)
            cont[f"{name}/file_size"] = np.int64(size)
            cont[f"{name}/parsed_json"] = np.frombuffer(json.dumps(md).encode(), np.uint8)
            assert bmd == blob and stg == fake
            k += 1
        # header overflow the reference raises on (struct.error): 2048^2 offsets / seglens
        with Quiet():
            for label, kw in (("big_offset", dict(start_offset=70000, segments_lengths=[1])),
                              ("neg_seglen", dict(start_offset=0, segments_lengths=[-1]))):
                try:
                    ref.create_header(codec="jxl", s=1, segments_indices=[0], bitmaps_blob_size=1, width=4,
                                      height=4, align_across_planes=False, **kw)
                    cont[f"err/{label}"] = np.array("none")
                except Exception as e:  # struct.error
                    cont[f"err/{label}"] = np.array(type(e).__name__)
    cont["__names__"] = np.array(["pe_b0.4_main", "torax_b0.4_1k", "ct12_37x53", "u8_5x5"])
    np.savez_compressed(os.path.join(HERE, "container.npz"), **cont)

    # --- DICOM files: header/trailer bytes around the pixel data (pixels are in images.npz)
    pe_raw = open(os.path.join(REF, "images", "pe.dcm"), "rb").read()
    tx_raw = open(os.path.join(REF, "images", "torax.dcm"), "rb").read()
    np.savez_compressed(os.path.join(HERE, "dicom_headers.npz"),
                        pe_head=np.frombuffer(pe_raw[:7010], np.uint8), pe_tail=np.frombuffer(pe_raw[7010 + 524288:], np.uint8),
                        torax_head=np.frombuffer(tx_raw[:888], np.uint8), torax_tail=np.frombuffer(tx_raw[888 + 262144:], np.uint8))


if __name__ == "__main__":
    main()
