# k_decide phase stamps at C3 (256 x 512^2 ct12; diagnostic build tools/bin/libcodec_hip_dts.so)
cd "$GRAFT_REPO_ROOT" || exit 9
DTS_B=256 DTS_SIZE=512 timeout -k 10 200 python tools/decide_phases.py ct12 2>&1 | grep -v amdgpu.ids
