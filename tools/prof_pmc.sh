#!/bin/bash
# PMC counters for one conv layer (pipe vs register-staged kernels); separate passes.
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
SHAPE=${SHAPE:-"96 128 512 512 3 16"}
for pipe in 1 0; do
  export DGVCC_CONV_PIPE=$pipe
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $OUT/p$pipe -o run -- python3 $R/tools/prof_conv_one.py $SHAPE fwd,wgrad > $OUT/log$pipe.txt 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$pipe -o run -- python3 $R/tools/prof_conv_one.py $SHAPE fwd,wgrad >> $OUT/log$pipe.txt 2>&1 || exit 1
done
