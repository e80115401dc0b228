# PMC passes over the C3 MED-PEE step (tools/c3_pee.py): issue stalls, clock and LDS behaviour
# of k_pee_embed_res (one pass per counter group; run from the repo root)
set -e
mkdir -p gpurun_out/res_pmc
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
    -d $R/gpurun_out/res_pmc/p3 -o run --output-format csv -- python3 $R/tools/c3_pee.py 5
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    -d $R/gpurun_out/res_pmc/p4 -o run --output-format csv -- python3 $R/tools/c3_pee.py 5
