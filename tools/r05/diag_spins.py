"""Stress the look-back's pixel-count fallback on the default grid at the headline shape:
CODEC_DEBUG=1 CODEC_PEE_LB_SPINS=<n> (tiny spin bound: most waits fall back) for the embed and
the extract, compared bit for bit with the default run."""
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    from codec_tcc_amd import synth
    from codec_tcc_amd.pee import PeeCodec
    B = int(os.environ.get("DIAG_B", "256"))
    H = W = 2048
    spins = sys.argv[1] if len(sys.argv) > 1 else "4"
    dev = torch.device("cuda", 0)
    covers = bench.make_covers(torch, "ct12", B, H, W, dev, 0)
    codec = PeeCodec(B, H, W, dtype="uint16", T=2, device=dev)
    packed = codec.pack_payloads([synth.payload(1024, 7 + i) for i in range(B)])
    pw = packed[0].shape[1]

    def setk(on):
        for k, v in (("CODEC_DEBUG", "1"), ("CODEC_PEE_LB_SPINS", spins)):
            if on:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)

    setk(False)
    ref = codec.embed(covers, None, stego=torch.empty_like(covers), packed=packed, check=False)
    wr, cr = codec.extract(ref.stego, ref.meta, ref.lm, payload_words=pw)
    wr, cr = wr.clone(), cr.clone()
    d0 = codec.diagnostics(pw)
    setk(True)
    for rep in range(3):
        alt = codec.embed(covers, None, stego=torch.empty_like(covers), packed=packed, check=False)
        wa, ca = codec.extract(ref.stego, ref.meta, ref.lm, payload_words=pw)
        torch.cuda.synchronize()
        sd = (alt.stego != ref.stego).flatten(1).any(1).sum().item()
        md = (alt.meta != ref.meta).flatten(1).any(1).sum().item()
        ld = (alt.lm != ref.lm).flatten(1).any(1).sum().item()
        cd = (ca != cr).flatten(1).any(1).sum().item()
        pd = (wa != wr).flatten(1).any(1).sum().item()
        print(f"spins={spins} rep {rep}: embed slices differing stego {sd} meta {md} map {ld}; "
              f"extract slices differing cover {cd} payload {pd}; diag {codec.diagnostics(pw)}", flush=True)
    setk(False)
    print("default restores the cover:", bool((cr == covers).all().item()), "diag at start", d0)


if __name__ == "__main__":
    main()
