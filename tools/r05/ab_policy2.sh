#!/bin/bash
export CODEC_TUNING=1   # CODEC_* knobs are honoured only under the tuning switch
# per-kernel cache policies (in-tree library, runtime knobs): the in-place slice-serial PEE
# passes' loads/stores (CODEC_PEE_IP_NTL / CODEC_PEE_IP_NTS) and C3's k_restore_il stores
# (CODEC_RIL_NTS), interleaved in one process; then the PEE and config GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/r05
timeout -k 10 400 python tools/tune_pee.py --modes ip --rounds 5 --configs '[{"CODEC_PEE_IP_NTL": "1", "CODEC_PEE_IP_NTS": "1"}, {"CODEC_PEE_IP_NTL": "1", "CODEC_PEE_IP_NTS": "0"}, {"CODEC_PEE_IP_NTL": "0", "CODEC_PEE_IP_NTS": "0"}, {"CODEC_PEE_IP_NTL": "0", "CODEC_PEE_IP_NTS": "1"}]' > gpurun_out/r05/ab_policy_ip.txt 2>&1 || { tail -5 gpurun_out/r05/ab_policy_ip.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05/ab_policy_ip.txt
timeout -k 10 300 python tools/tune.py --size 512 --rounds 7 --steps 20 --configs '[{"CODEC_RIL_NTS": "1"}, {"CODEC_RIL_NTS": "0"}]' > gpurun_out/r05/ab_policy_ril.txt 2>&1 || { tail -5 gpurun_out/r05/ab_policy_ril.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05/ab_policy_ril.txt
timeout -k 10 600 python -u -m pytest tests/test_pee.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_policy.log 2>&1; rc=$?
tail -3 gpurun_out/r05/pytest_policy.log; exit $rc
