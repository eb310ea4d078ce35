#!/bin/bash
# 64->64 3x3 conv at 768x1024 (B=16): kernel trace for both 3-tap K widths, then SQ/TCC
# counter passes on the default build.  Every step has its own time limit.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/diag_tap3
mkdir -p $OUT
ARGS="768 1024 64 64 3 16 ${KINDS:-fwd,dgrad}"
for bk in 64 32; do
  DGVCC_TAP3_BK=$bk timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bk$bk -o run -- python3 tools/prof_conv_one.py $ARGS > $OUT/bk$bk.log 2>&1 || exit $?
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- python3 tools/prof_conv_one.py $ARGS > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_tcc -o run -- python3 tools/prof_conv_one.py $ARGS > $OUT/tcc.log 2>&1 || exit $?
echo done
