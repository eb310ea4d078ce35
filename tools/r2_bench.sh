#!/bin/bash
# Round-2 measurement of the headline workload (bench.py defaults: sta_final final mode,
# fp32, + the bf16 leg and the CPU baseline), then rocprofv3 kernel stats, PMC HBM traffic
# and MFMA-busy passes for both precisions.  Usage: PROF_TAG=r2a bash tools/r2_bench.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-r2}
mkdir -p $OUT
ONLY=${ONLY:-all}
if [ "$ONLY" = all ] || [ "$ONLY" = bench ]; then
  timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
F32="--steps 2 --warmup 1 --no-cpu-baseline --no-bf16 --no-f32-exact"
B16="--steps 5 --warmup 2 --no-cpu-baseline --precision bf16 --no-f32-exact"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_fp32 -o run -- python3 bench.py $F32 > $OUT/trace_fp32.json 2> $OUT/trace_fp32.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bf16 -o run -- python3 bench.py $B16 > $OUT/trace_bf16.json 2> $OUT/trace_bf16.err || exit $?
P1="--steps 1 --warmup 1 --no-cpu-baseline --no-f32-exact"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_fp32 -o run -- python3 bench.py $P1 --no-bf16 > /dev/null 2> $OUT/pmc1.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_fp32 -o run -- python3 bench.py $P1 --no-bf16 > /dev/null 2> $OUT/pmc2.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_bf16 -o run -- python3 bench.py $P1 --precision bf16 > /dev/null 2> $OUT/pmc3.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_bf16 -o run -- python3 bench.py $P1 --precision bf16 > /dev/null 2> $OUT/pmc4.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma_fp32 -o run -- python3 bench.py $P1 --no-bf16 > /dev/null 2> $OUT/pmc5.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma_bf16 -o run -- python3 bench.py $P1 --precision bf16 > /dev/null 2> $OUT/pmc6.err || exit $?
echo done
