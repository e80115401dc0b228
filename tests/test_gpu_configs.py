"""BASELINE.json configs through the default launch shapes the benchmark uses:

* C3 -- 256 x 512^2 slices on one GPU;
* the headline shape -- 256 x 2048^2 (k_scan_rows, k_decide_embed, k_restore_gs for the
  reference's LSB path; k_pee_embed1 / k_pee_extract1 lane-order single pass for MED-PEE).

Each batch is compared with the oracles on a stride sample of slices (s, start offset,
stego; PEE stego, location map, end), the reference's own 2048^2 known answers are placed
as slices inside the headline batch, and every slice is checked by exact round trip
(restored cover and recovered payload bits).  Covers are generated on the device
(synth.ct12_torch); the sampled slices are copied back for the oracle."""
import hashlib
import os
import sys

import numpy as np
import pytest

import golden_io
from codec_tcc_amd import Codec, framing, make_payloads, synth
from oracle import pee_cpu as P
from oracle import ref_cpu as R

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import payload_equal  # noqa: E402

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _batch(B, H, W, seed):
    return synth.ct12_torch(B, H, W, "cuda", seed=seed).view(torch.uint16)


def _lsb_batch_check(covers, msgs, sample, kats=()):
    B, H, W = covers.shape
    codec = Codec(B, H, W, dtype="uint16", beta=0.4, block=16)
    pl = make_payloads(msgs, covers.device)
    enc = codec.encode(covers, pl)
    recs = enc.records()
    for i in sample:
        cov = covers[i].cpu().numpy()
        exp = R.encode_slice(cov, R.message_to_bits(msgs[i]), beta=0.4, sb=16)
        assert recs[i].s == exp["s"] and recs[i].start_offset == exp["start_offset"], i
        assert [recs[i].perm[j] for j in range(exp["s"])] == list(exp["segment_indices"])
        np.testing.assert_array_equal(enc.stego[i].cpu().numpy(), exp["stego"])
    for i, kat in kats:
        m = recs[i]
        assert m.s == kat["s"] and [m.perm[j] for j in range(m.s)] == kat["perm"]
        assert [m.sizes[p] for p in range(m.s)] == kat["sizes"]
        assert hashlib.sha256(enc.stego[i].cpu().numpy().tobytes()).hexdigest() == kat["stego_sha256"]
    words, cover = codec.decode(enc.stego, enc.maps, enc.meta, payload_words=pl.payload_words,
                                map_words=pl.map_words)
    assert torch.equal(cover.view(torch.int16), covers.view(torch.int16))
    assert all(r.total_used == n and r.status == 0 for r, n in zip(recs, pl.lengths))
    assert payload_equal(words, pl.words, pl.lengths)


def _pee_batch_check(covers, sample, T=2, chars=1024):
    from codec_tcc_amd.pee import PeeCodec, lm_bits
    B, H, W = covers.shape
    codec = PeeCodec(B, H, W, dtype="uint16", T=T)
    payloads = [framing.to_bits(synth.payload(chars, 300 + i)) for i in range(B)]
    packed = codec.pack_payloads(payloads)
    enc = codec.embed(covers, None, packed=packed)
    recs = enc.records()
    t_dev = codec.t_slices.cpu().numpy() if T == "auto" else None
    for i in sample:
        cov = covers[i].cpu().numpy()
        Ti = P.select_T(cov, len(payloads[i]), codec.tmax) if T == "auto" else T
        assert recs[i].T == Ti
        if t_dev is not None:
            assert t_dev[i] == Ti, i
        st, side = P.pee_embed(cov, payloads[i], Ti)
        assert recs[i].status == 0 and recs[i].end == side["end"], i
        np.testing.assert_array_equal(enc.stego[i].cpu().numpy(), st)
        np.testing.assert_array_equal(lm_bits(enc, i), side["lm"])
    words, cover = codec.extract(enc.stego, enc.meta, enc.lm, payload_words=enc.payload_words)
    assert torch.equal(cover.view(torch.int16), covers.view(torch.int16))
    assert all(r.status == 0 for r in recs) and not codec.lookback_failed(enc.payload_words)
    assert payload_equal(words, packed[0], [len(p) for p in payloads])
    assert codec.repaired(enc.payload_words) == 0
    # in place on the same batch: the stego and the payload equal the out-of-place ones
    work = covers.clone()
    enc2 = codec.embed(work, None, stego=work, packed=packed)
    assert torch.equal(work.view(torch.int16), enc.stego.view(torch.int16))
    w2, _ = codec.extract(work, enc2.meta, enc2.lm, payload_words=enc2.payload_words, cover=work)
    assert torch.equal(work.view(torch.int16), covers.view(torch.int16))
    assert payload_equal(w2, packed[0], [len(p) for p in payloads])


def test_c3_lsb_256x512():
    B, H, W = 256, 512, 512
    covers = _batch(B, H, W, seed=1000)
    msgs = [synth.payload(1024, 5000 + i) for i in range(B)]
    _lsb_batch_check(covers, msgs, sample=range(0, B, 16))


@pytest.mark.parametrize("ss", ["auto", "res0", "0", "unfused"])
def test_c3_pee_256x512(ss, monkeypatch):
    """1 KB per 512^2 ct12 slice needs T ~ 4-5 (T = 2 holds ~4.4 kbit): capacity control.
    "auto": the default launch, the resident embed (k_pee_embed_res: the slice read once and
    kept on the CU while T is chosen); "res0": capacity fused into the two-phase slice-serial
    embed (CODEC_PEE_RES=0); "unfused": capacity pass + slice-serial embed as two launches;
    "0": capacity pass + look-back embed."""
    if ss == "unfused":
        monkeypatch.setenv("CODEC_PEE_AUTO_FUSED", "0")
    elif ss == "res0":
        monkeypatch.setenv("CODEC_PEE_RES", "0")
    elif ss != "auto":
        monkeypatch.setenv("CODEC_PEE_SS", ss)
    _pee_batch_check(_batch(256, 512, 512, seed=2000), sample=range(3, 256, 16), T="auto")


def test_headline_lsb_256x2048_with_kats():
    """The bench's launch shape, the reference's 2048^2 known answers (beta 0.4) as slices
    37 and 200 of the batch, oracle comparison on 4 more slices."""
    B, H, W = 256, 2048, 2048
    covers = _batch(B, H, W, seed=0)
    msgs = [synth.payload(1024, 7 + i) for i in range(B)]
    kats = []
    for pos, kat in zip((37, 200), [k for k in golden_io.kat2048() if k["beta"] == 0.4]):
        img = synth.GENERATORS[kat["kind"]](kat["h"], kat["w"], kat["seed"])
        assert hashlib.sha256(img.tobytes()).hexdigest() == kat["cover_sha256"]
        covers[pos].copy_(torch.from_numpy(img).view(torch.uint16))
        msgs[pos] = synth.payload(kat["payload_chars"], kat["payload_seed"])
        kats.append((pos, kat))
    assert len(kats) == 2
    _lsb_batch_check(covers, msgs, sample=(0, 85, 170, 255), kats=kats)


@pytest.mark.parametrize("ss", ["auto", "1"])
def test_headline_pee_256x2048(ss, monkeypatch):
    """Default dispatch at this shape (codec_pee.hip pee_use_slice_serial): out of place the
    look-back single pass (k_pee_embed1 / k_pee_extract1, chunk-parallel), in place the
    slice-serial pass (k_pee_embed_ss / k_pee_extract_ss).  "1" forces the slice-serial
    kernels out of place too, so the out-of-place k_pee_embed_ss runs once at 2048^2."""
    if ss != "auto":
        monkeypatch.setenv("CODEC_PEE_SS", ss)
    _pee_batch_check(_batch(256, 2048, 2048, seed=11), sample=(0, 101, 255))
