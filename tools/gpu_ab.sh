#!/bin/bash
# Development round trip: the GPU tests, then a rocprofv3 kernel-trace of a short bench
# (per-kernel averages to compare against profiles/<round>/kernel_stats_bench_b16.csv).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc"; tail -30 gpurun_out/tests.log; exit $rc; fi
OUT=gpurun_out/${PROF_TAG:-ab}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} > $OUT/bench_trace.json 2> $OUT/trace.err || exit $?
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
