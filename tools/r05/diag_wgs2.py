"""Which pass goes wrong under a persistent grid (CODEC_PEE_1P_WGS) at the headline shape:
embed with the knob vs the default embed (stego / meta / map, per slice), then each extract."""
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    from codec_tcc_amd import synth
    from codec_tcc_amd.pee import PeeCodec
    B = int(os.environ.get("DIAG_B", "256"))
    H = W = 2048
    wgs = sys.argv[1] if len(sys.argv) > 1 else "2048"
    dev = torch.device("cuda", 0)
    covers = bench.make_covers(torch, "ct12", B, H, W, dev, 0)
    codec = PeeCodec(B, H, W, dtype="uint16", T=2, device=dev)
    packed = codec.pack_payloads([synth.payload(1024, 7 + i) for i in range(B)])

    def embed(knob):
        if knob:
            os.environ["CODEC_PEE_1P_WGS"] = knob
        else:
            os.environ.pop("CODEC_PEE_1P_WGS", None)
        st = torch.empty_like(covers)
        e = codec.embed(covers, None, stego=st, packed=packed, check=False)
        torch.cuda.synchronize()
        return e

    def extract(e, knob):
        if knob:
            os.environ["CODEC_PEE_1P_WGS"] = knob
        else:
            os.environ.pop("CODEC_PEE_1P_WGS", None)
        w, c = codec.extract(e.stego, e.meta, e.lm, payload_words=e.payload_words)
        torch.cuda.synchronize()
        return w.clone(), c.clone()

    d0 = codec.diagnostics(packed[0].shape[1])
    ref = embed(None)
    alt = embed(wgs)
    d1 = codec.diagnostics(packed[0].shape[1])
    sdiff = (ref.stego != alt.stego).flatten(1).sum(1).cpu().numpy()
    mdiff = (ref.meta != alt.meta).flatten(1).sum(1).cpu().numpy()
    ldiff = (ref.lm != alt.lm).flatten(1).sum(1).cpu().numpy()
    print("embed WGS=%s vs default: slices with stego diffs %d (px %d), meta diffs %d, map diffs %d" % (
        wgs, (sdiff > 0).sum(), sdiff.sum(), (mdiff > 0).sum(), (ldiff > 0).sum()))
    print("  diag before", d0, "after", d1)
    bad = np.nonzero(sdiff)[0][:8]
    print("  first bad slices", bad.tolist(), "px", sdiff[bad].tolist())
    wr, cr = extract(ref, None)
    wa, ca = extract(ref, wgs)
    print("extract WGS=%s of the default stego: cover diffs in %d slices, payload diffs in %d slices" % (
        wgs, ((cr != ca).flatten(1).sum(1) > 0).sum().item(), ((wr != wa).flatten(1).sum(1) > 0).sum().item()))
    print("  default extract restores the cover:", bool((cr == covers).all().item()))
    print("  diag now", codec.diagnostics(packed[0].shape[1]))


if __name__ == "__main__":
    main()
