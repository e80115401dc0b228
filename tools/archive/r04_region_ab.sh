# A/B: k_restore_gs streaming contiguous per-workgroup regions (CODEC_RESTORE_GS_REGION
# workgroups) against its grid-stride sweep -- headline 256 x 2048^2 and C2 1 x 2048^2
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/tune.py --rounds 4 --steps 5 --configs '[{},{"CODEC_RESTORE_GS_REGION":"512","CODEC_RESTORE_GS_THREADS":"1024"},{"CODEC_RESTORE_GS_REGION":"1024","CODEC_RESTORE_GS_THREADS":"1024"},{"CODEC_RESTORE_GS_REGION":"2048","CODEC_RESTORE_GS_THREADS":"1024"},{"CODEC_RESTORE_GS_REGION":"4096","CODEC_RESTORE_GS_THREADS":"1024"},{"CODEC_RESTORE_GS_REGION":"1024","CODEC_RESTORE_GS_THREADS":"256"},{"CODEC_RESTORE_GS_REGION":"4096","CODEC_RESTORE_GS_THREADS":"256"},{"CODEC_RESTORE_GS_REGION":"1024","CODEC_RESTORE_GS_THREADS":"1024"}]' > gpurun_out/region_ab.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/tune.py --batch 1 --rounds 4 --steps 10 --configs '[{},{"CODEC_RESTORE_GS_REGION":"256"},{"CODEC_RESTORE_GS_REGION":"512","CODEC_RESTORE_GS_THREADS":"256"},{"CODEC_RESTORE_GS_REGION":"128"}]' > gpurun_out/region_ab_c2.log 2>&1
