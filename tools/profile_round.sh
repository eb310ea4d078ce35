#!/bin/bash
# rocprofv3 kernel-trace stats + PMC HBM traffic passes for bench.py (default workload).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/write.err || exit $?
echo done
