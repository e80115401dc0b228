"""The A/B knobs' tuning switch (include/codec_tcc.h, codec_set_tuning).

With the switch off -- the product default -- the CODEC_* environment variables that pick
launch shapes are ignored: the default kernels run and the results are those of the default
path.  With it on (this suite turns it on in conftest.py) the same variables do change the
kernels, and the results stay identical (every knob is a launch-shape choice, not a
semantic one)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

KNOBS = {"CODEC_PEE_SS": "1", "CODEC_SCAN_KIND": "0", "CODEC_FUSED_DECIDE": "0", "CODEC_DECIDE_EXACT": "1",
         "CODEC_HIST_MEMSET": "1"}


def _tagged(lib, _lib, fn):
    """fn()'s result and the sorted kernel tags its launches recorded (codec_profile_*)."""
    cap = 256
    _lib.check(lib.codec_profile_begin(cap), "codec_profile_begin")
    out = fn()
    torch.cuda.synchronize()
    ms = (C.c_float * cap)()
    tags = (C.c_int32 * cap)()
    n = lib.codec_profile_end(ms, tags, cap)
    return out, sorted({_lib.KERNEL_TAGS.get(tags[i], str(tags[i])) for i in range(max(n, 0))})


def _snapshot(lsb, pee):
    return [lsb.stego.view(torch.int16).cpu().numpy(), lsb.maps.cpu().numpy(), lsb.meta.cpu().numpy(),
            pee.stego.view(torch.int16).cpu().numpy(), pee.lm.cpu().numpy(), pee.meta.cpu().numpy()]


def test_knobs_ignored_without_tuning(monkeypatch):
    import bench
    import codec_tcc_amd as ct
    from codec_tcc_amd import _lib, synth
    from codec_tcc_amd.pee import PeeCodec
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    B, H, W = 256, 512, 512                     # chip-filling: the fused LSB scan + decision
    covers = bench.make_covers(torch, "ct12", B, H, W, dev, seed=4242)
    codec = ct.Codec(B, H, W, dtype="uint16", beta=0.4, block=16, device=dev)
    pl = ct.make_payloads([synth.payload(1024, 77 + i) for i in range(B)], dev)
    pb = 8                                      # a small out-of-place batch: the look-back MED-PEE pass
    pee = PeeCodec(pb, H, W, dtype="uint16", T=2, device=dev)
    pcov = covers[:pb].contiguous()
    pmsg = [synth.payload(800, 300 + i) for i in range(pb)]

    def run():
        return codec.encode(covers, pl), pee.embed(pcov, pmsg)

    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    ref, ref_tags = _tagged(lib, _lib, run)
    assert "k_scan_decide" in ref_tags and "k_pee_embed1" in ref_tags, ref_tags
    assert all(r.flags & _lib.FLAG_INFO_FAST for r in ref[0].records())
    want = _snapshot(*ref)

    for k, v in KNOBS.items():
        monkeypatch.setenv(k, v)
    prev = lib.codec_set_tuning(0)
    try:
        got, got_tags = _tagged(lib, _lib, run)
    finally:
        lib.codec_set_tuning(prev)
    assert prev == 1
    assert got_tags == ref_tags                  # the default kernels ran
    assert all(r.flags & _lib.FLAG_INFO_FAST for r in got[0].records())   # CODEC_DECIDE_EXACT ignored
    for a, b in zip(_snapshot(*got), want):
        np.testing.assert_array_equal(a, b)

    # the switch on: the same variables now pick other kernels, with identical results
    alt, alt_tags = _tagged(lib, _lib, run)
    assert "k_scan_decide" not in alt_tags and "k_pee_embed_ss" in alt_tags, alt_tags
    assert not any(r.flags & _lib.FLAG_INFO_FAST for r in alt[0].records())
    snap = _snapshot(*alt)
    for i in (0, 1, 3, 4):
        np.testing.assert_array_equal(snap[i], want[i])
    for r, q in zip(alt[1].records(), ref[1].records()):   # MED-PEE meta (capacity/PARTIAL are path-specific)
        assert (r.T, r.L, r.end, r.nc, r.lm_count, r.status) == (q.T, q.L, q.end, q.nc, q.lm_count, q.status)
    for r, q in zip(alt[0].records(), ref[0].records()):   # LSB meta: same decision, exact info
        assert (r.s, r.start_offset, r.total_used, r.entropy) == (q.s, q.start_offset, q.total_used, q.entropy)
