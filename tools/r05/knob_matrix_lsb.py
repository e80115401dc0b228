"""LSB (the reference's path) launch knobs against the default path (round 5 audit): each
configuration's encode (stego, maps, meta) and decode (payload words, restored cover) must equal
the default run's bit for bit, at the headline slice size (DIAG_B x 2048^2) and at C3 (256 x 512^2).
ct12 slices, 1 KB payloads."""
import json
import os
os.environ.setdefault("CODEC_TUNING", "1")   # the library honours CODEC_* knobs only under this switch
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

CONFIGS = [
    {"CODEC_SCAN_KIND": "0"},
    {"CODEC_DECIDE_WAVES": "0"},
    {"CODEC_DECIDE_PAIRS": "0"},
    {"CODEC_DECIDE_SPLIT": "0"},
    {"CODEC_FUSED_DECIDE": "0"},
    {"CODEC_FUSED_EMBED": "0"},
    {"CODEC_FUSED_GATHER": "0"},
    {"CODEC_RESTORE_GS": "0"},
    {"CODEC_RESTORE_IL": "0"},
    {"CODEC_RESTORE_SS": "1"},
    {"CODEC_RIL_NTS": "1"},
    {"CODEC_NT": "0"},
    {"CODEC_HIST_MEMSET": "1"},
]


def main():
    import torch
    import bench
    import codec_tcc_amd as ct
    from codec_tcc_amd import synth
    dev = torch.device("cuda", 0)
    bad = 0
    for B, S in ((int(os.environ.get("DIAG_B", "32")), 2048), (256, 512)):
        covers = bench.make_covers(torch, "ct12", B, S, S, dev, 9)
        codec = ct.Codec(B, S, S, dtype="uint16", device=dev)
        pl = ct.make_payloads([synth.payload(1024, 50 + i) for i in range(B)], dev)

        def run():
            e = codec.encode(covers, pl, check=False)
            words, cov = codec.decode(e.stego, e.maps, e.meta, payload_words=pl.payload_words, map_words=pl.map_words)
            torch.cuda.synchronize()
            return e.stego.clone(), e.maps.clone(), e.meta.clone(), words.clone(), cov.clone()

        ref = run()
        assert torch.equal(ref[4], covers), "default decode does not restore the cover"
        for cfg in CONFIGS:
            saved = {k: os.environ.get(k) for k in cfg}
            os.environ.update(cfg)
            got = run()
            names = ["stego", "maps", "meta", "payload", "cover"]
            diff = [n for n, a, b in zip(names, got, ref) if not torch.equal(a, b)]
            bad += bool(diff)
            print(json.dumps({"shape": [B, S, S], "cfg": cfg, "diff": diff}), flush=True)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    print("configs with differences:", bad)


if __name__ == "__main__":
    main()
