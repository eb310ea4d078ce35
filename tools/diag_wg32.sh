#!/bin/bash
# fp32 wgrad / fwd of one 256->256 3x3 layer at 192x256 (B=16): kernel trace + SQ counters.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-diag_wg32}
mkdir -p $OUT
export DGVCC_PROF_DT=f32
ARGS="192 256 256 256 3 16 ${KINDS:-fwd,wgrad}"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_conv_one.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- python3 tools/prof_conv_one.py $ARGS > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq2 -o run -- python3 tools/prof_conv_one.py $ARGS > $OUT/sq2.log 2>&1 || exit $?
echo done
