#!/bin/bash
# Round-2 baseline: GPU tests, then the final-mode step in fp32 and bf16 with kernel stats.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-r2base}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 bench.py --mode final --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/final_fp32.json 2> $OUT/final_fp32.err || { echo "fp32 bench failed"; tail -20 $OUT/final_fp32.err; exit 1; }
cat $OUT/final_fp32.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace32 -o run -- python3 bench.py --mode final --precision fp32 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace32.json 2> $OUT/trace32.err || exit $?
timeout -k 10 300 python3 bench.py --mode final --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/final_bf16.json 2> $OUT/final_bf16.err || { echo "bf16 bench failed"; tail -20 $OUT/final_bf16.err; exit 1; }
cat $OUT/final_bf16.json
echo done
