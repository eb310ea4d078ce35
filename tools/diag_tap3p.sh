#!/bin/bash
# tap3p diagnosis: full kernel vs no-MFMA vs no-strip-DMA variants on the 64->64 768x1024 layer.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/diag_tap3p
mkdir -p $OUT
for d in 0 1 2; do
  DGVCC_TAP3P_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dbg$d -o run -- python3 tools/prof_conv_one.py 768 1024 64 64 3 16 fwd > $OUT/dbg$d.log 2>&1 || exit $?
  grep -h tap3p $OUT/dbg$d/run_kernel_stats.csv | cut -d, -f1-4
done
