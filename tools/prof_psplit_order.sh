#!/bin/bash
# HBM fetch and time of the f32 pre-split forward on one layer under both tile walks
# (DGVCC_PSPLIT_ORDER=0: pixel-major, both filter panels on every XCD; =1: channel-major, each
# XCD's tiles share one panel).  usage: PROF_TAG=x [SHAPE="96 128 512 512 3 32"] bash tools/prof_psplit_order.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-order}; mkdir -p $OUT
SHAPE=${SHAPE:-"96 128 512 512 3 32"}
for O in 0 1; do
  DGVCC_PROF_DT=f32 DGVCC_PSPLIT_ORDER=$O timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$O -o run -- python3 tools/prof_conv_one.py $SHAPE fwd > $OUT/t$O.log 2>&1 || exit 1
  DGVCC_PROF_DT=f32 DGVCC_PSPLIT_ORDER=$O timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f$O -o run -- python3 tools/prof_conv_one.py $SHAPE fwd > $OUT/f$O.log 2>&1 || exit 1
  DGVCC_PROF_DT=f32 DGVCC_PSPLIT_ORDER=$O timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/h$O -o run -- python3 tools/prof_conv_one.py $SHAPE fwd > $OUT/h$O.log 2>&1 || exit 1
done
echo ok
