#!/bin/bash
# Round-4 evidence run: (optionally) the GPU tests, the default bench line (cpu_baseline + parity
# legs included), smoke, then the headline-only (fp32) and bf16 rocprofv3 passes of
# tools/prof_headline.sh.  PROF_TAG names the gpurun_out/ directory; SKIP_TESTS=1 skips pytest.
set -u
TAG=${PROF_TAG:-r4}
mkdir -p gpurun_out/$TAG
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
  tail -1 gpurun_out/$TAG/tests.log
fi
timeout -k 10 600 python3 -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
tail -c 400 gpurun_out/$TAG/bench.json
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
if [ "${SKIP_PROF:-0}" != "1" ]; then
  PROF_TAG=$TAG/hl bash tools/prof_headline.sh || exit 1
  BENCH_EXTRA="--precision bf16" PROF_TAG=$TAG/bf16 bash tools/prof_headline.sh || exit 1
fi
echo ok
