#!/bin/bash
# GPU test suite (one process, per-test timeouts).  Usage: PROF_TAG=t1 bash tools/r2_tests.sh [pytest args]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-tests}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread "$@" > $OUT/tests.log 2>&1
rc=$?
tail -40 $OUT/tests.log
exit $rc
