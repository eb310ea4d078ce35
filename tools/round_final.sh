#!/bin/bash
# End-of-round measurement: GPU tests, the default bench line (with cpu_baseline and
# parity), rocprofv3 kernel stats, PMC HBM traffic and MFMA-busy passes.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${PROF_TAG:-final}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
PROF_TAG=$TAG bash tools/profile_round.sh || exit $?
PROF_TAG=$TAG bash tools/prof_mfma.sh || exit $?
