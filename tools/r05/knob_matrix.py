"""MED-PEE launch knobs at the headline slice size, against the default path (round 5 audit,
after the persistent-grid bug): each configuration's embed (stego, meta, map) and extract
(payload words, restored cover) must equal the default run's bit for bit, out of place and in
place.  DIAG_B slices of 2048^2 ct12, T = 2, 1 KB payloads."""
import json
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

CONFIGS = [{"CODEC_PEE_ONEPASS": "0"}] if os.environ.get("ONLY_TWOPASS") else [
    {"CODEC_PEE_1P_NOTICKET": "0", "CODEC_PEE_X_NOTICKET": "0"},
    {"CODEC_PEE_1P_CHUNK_MAJOR": "0"},
    {"CODEC_PEE_1P_GROUP": "8", "CODEC_PEE_X_GROUP": "8"},
    {"CODEC_PEE_1P_GROUP": "64", "CODEC_PEE_X_GROUP": "64"},
    {"CODEC_PEE_1P_WGS": "768"},
    {"CODEC_PEE_1P_WGS": "2048"},
    {"CODEC_PEE_ONEPASS": "0"},
    {"CODEC_PEE_SS": "1"},
    {"CODEC_PEE_SS": "0"},
    {"CODEC_PEE_IP_WGS": "512"},
    {"CODEC_PEE_IP_WGS": "8192"},
    {"CODEC_PEE_SS_D": "2", "CODEC_PEE_SSX_D": "6"},
    {"CODEC_PEE_IP_NTS": "1", "CODEC_PEE_IP_NTL": "0"},
    {"CODEC_NT": "0"},
]


def main():
    import torch
    import bench
    from codec_tcc_amd import synth
    from codec_tcc_amd.pee import PeeCodec
    B = int(os.environ.get("DIAG_B", "64"))
    H = W = 2048
    dev = torch.device("cuda", 0)
    covers = bench.make_covers(torch, "ct12", B, H, W, dev, 5)
    codec = PeeCodec(B, H, W, dtype="uint16", T=2, device=dev)
    packed = codec.pack_payloads([synth.payload(1024, 31 + i) for i in range(B)])
    pw = packed[0].shape[1]

    def run(inplace):
        if inplace:
            st = covers.clone()
            e = codec.embed(st, None, stego=st, packed=packed, check=False)
        else:
            e = codec.embed(covers, None, stego=torch.empty_like(covers), packed=packed, check=False)
        stego = e.stego.clone()
        if inplace:   # the restored cover overwrites the stego
            words, cov = codec.extract(e.stego, e.meta, e.lm, payload_words=pw, cover=e.stego)
        else:
            words, cov = codec.extract(e.stego, e.meta, e.lm, payload_words=pw)
        torch.cuda.synchronize()
        return stego, e.meta.clone(), e.lm.clone(), words.clone(), cov.clone()

    ref = {m: run(m) for m in (False, True)}
    assert torch.equal(ref[False][4], covers), "default out-of-place extract does not restore the cover"
    bad = 0
    for cfg in CONFIGS:
        saved = {k: os.environ.get(k) for k in cfg}
        os.environ.update(cfg)
        for m in (False, True):
            got = run(m)
            names = ["stego", "meta", "map", "payload", "cover"]
            diff = [n for n, a, b in zip(names, got, ref[m]) if not torch.equal(a, b)]
            if "meta" in diff:   # which record fields differ
                from codec_tcc_amd import _lib
                def recs(t):
                    raw = t.cpu().contiguous().numpy().tobytes()
                    return [_lib.PeeMeta.from_buffer_copy(raw, i * _lib.PEE_META_BYTES) for i in range(B)]
                ra, rb = recs(got[1]), recs(ref[m][1])
                fields = sorted({f for a, b in zip(ra, rb) for f, _ in _lib.PeeMeta._fields_
                                 if str(getattr(a, f)) != str(getattr(b, f))})
                diff.append("meta fields: " + ",".join(fields))
                fa = fields[0] if fields else None
                if fa:
                    diff.append("e.g. slice 0 %s: %s vs default %s" % (fa, getattr(ra[0], fa), getattr(rb[0], fa)))
            if m:   # in place must also match the out-of-place stego
                if not torch.equal(got[0], ref[False][0]):
                    diff.append("stego vs out-of-place")
            bad += bool(diff)
            print(json.dumps({"cfg": cfg, "inplace": m, "diff": diff, "diag": codec.diagnostics(pw)}), flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    print("configs with differences:", bad)


if __name__ == "__main__":
    main()
