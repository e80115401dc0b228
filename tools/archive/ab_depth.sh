cd "$GRAFT_REPO_ROOT"
for i in 1 2; do for d in 4 2; do
CODEC_PEE_SS_D=$d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --lsb 0 --c2 0 --c3 0 --cpu-seconds 0 > gpurun_out/d$d.json 2>gpurun_out/d$d.err || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/d$d.json').read().strip().splitlines()[-1]);ip=d['inplace'];print('D=$d',ip['ms_per_step'],ip['kernels_ms'],ip['roofline']['frac'],ip['roundtrip_ok'])"
done; done
