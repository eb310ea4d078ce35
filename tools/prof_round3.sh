#!/bin/bash
# Round-3 evidence run: GPU tests, the default bench line (cpu_baseline + parity legs included),
# then the headline-only (fp32) and bf16 rocprofv3 passes of tools/prof_headline.sh.
set -u
TAG=${PROF_TAG:-r3final}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
tail -c 400 gpurun_out/$TAG/bench.json
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
PROF_TAG=$TAG/hl bash tools/prof_headline.sh || exit 1
BENCH_EXTRA="--precision bf16" PROF_TAG=$TAG/bf16 bash tools/prof_headline.sh || exit 1
echo ok
