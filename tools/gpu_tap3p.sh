#!/bin/bash
# persistent 3-tap kernel: parity tests, then same-box A/B of the default bench and a kernel trace.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tap3p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "tap3 or persistent" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do DGVCC_TAP3P_ROWS=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$r -o run -- python3 tools/prof_conv_one.py 768 1024 64 64 3 16 fwd,dgrad > $OUT/one$r.log 2>&1 || exit $?; done
AB_VARS="DGVCC_TAP3P=0 DGVCC_TAP3P_ROWS=1 DGVCC_TAP3P_ROWS=2 DGVCC_TAP3P=0 DGVCC_TAP3P_ROWS=1 DGVCC_TAP3P_ROWS=2" bash tools/ab_env.sh || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/all_tests.log 2>&1 || { echo "gpu suite failed"; tail -30 $OUT/all_tests.log; exit 1; }
tail -1 $OUT/all_tests.log
