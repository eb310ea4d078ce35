#!/bin/bash
# tap3p counted-vmcnt tile boundary: parity tests, standalone layer A/B and bench A/B.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/cnt
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "tap3 or persistent or eval" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 0 1; do
  DGVCC_TAP3P_CNT=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cnt$c -o run -- python3 tools/prof_conv_one.py 768 1024 64 64 3 16 fwd,dgrad > $OUT/cnt$c.log 2>&1 || exit $?
  grep -h tap3p $OUT/cnt$c/run_kernel_stats.csv | cut -d, -f1-4
done
AB_VARS="DGVCC_TAP3P_CNT=0 DGVCC_TAP3P_CNT=1 DGVCC_TAP3P_CNT=0 DGVCC_TAP3P_CNT=1" bash tools/ab_env.sh || exit $?
