#!/bin/bash
# GPU round-trip used during development: gpu tests, then (only if they did not
# crash) a short bench.  Every GPU step has its own time limit.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/tests.log
if [ $rc -gt 1 ]; then echo "tests crashed/timed out rc=$rc"; exit $rc; fi
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  brc=$?
  echo "bench rc=$brc"
  exit $brc
fi
exit $rc
