# slice-serial vs look-back MED-PEE on one box: GPU tests, phase trace, bench legs
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_pee.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ss.log 2>&1; rc=$?; tail -2 gpurun_out/ss.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/ss_trace.py run inplace > gpurun_out/trace_ip.txt 2>&1 || exit 4
head -8 gpurun_out/trace_ip.txt
for ss in 1 0; do CODEC_PEE_SS=$ss timeout -k 10 200 python bench.py --lsb 0 --c2 0 --cpu-seconds 0 --steps 20 > gpurun_out/b_ss$ss.json 2>gpurun_out/b_ss$ss.err || exit 3; done
python - <<PY
import json
for ss in ("1","0"):
    d=json.loads(open("gpurun_out/b_ss%s.json"%ss).read().strip().splitlines()[-1])
    print(ss, d["value"], d["ms_per_step"], d["kernels_ms"], d["roundtrip_ok"], "inplace", d["inplace"]["ms_per_step"], d["inplace"]["kernels_ms"], d["inplace"]["roundtrip_ok"], "c3", d["c3"]["ms_per_step"], d["c3"]["kernels_ms"])
PY
