#!/bin/bash
# f32 split-math check: conv kernel + model parity tests, then the fp32 final-mode step with
# the split (default) and exact f32 MFMA arithmetic.  Usage: PROF_TAG=s1 bash tools/r2_split.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-split}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
B="--steps 3 --warmup 1 --no-cpu-baseline --no-bf16 --no-f32-exact"
timeout -k 10 300 python3 bench.py $B > $OUT/bench_split.json 2> $OUT/bench_split.err || { tail -20 $OUT/bench_split.err; exit 1; }
cat $OUT/bench_split.json
DGVCC_PSPLIT=0 timeout -k 10 300 python3 bench.py $B > $OUT/bench_exact.json 2> $OUT/bench_exact.err || { tail -20 $OUT/bench_exact.err; exit 1; }
cat $OUT/bench_exact.json
