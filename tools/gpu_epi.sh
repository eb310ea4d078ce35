#!/bin/bash
# LDS-staged epilogue constants: parity tests, the GPU suite, bench x2 and a kernel trace.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/epi
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "tap3 or persistent or eval" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/all_tests.log 2>&1 || { echo "gpu suite failed"; tail -30 $OUT/all_tests.log; exit 1; }
tail -1 $OUT/all_tests.log
AB_VARS="DGVCC_X=0 DGVCC_Y=0" bash tools/ab_env.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err || exit $?
grep -E "pers_kernel|tap3|wgrad9" $OUT/trace/run_kernel_stats.csv | cut -d, -f1-4
