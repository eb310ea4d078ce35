#!/bin/bash
# One bench.py configuration profiled for tools/step_table.py: kernel trace, then separate PMC
# passes for HBM bytes (FETCH_SIZE, WRITE_SIZE) and MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES +
# GRBM_GUI_ACTIVE).  usage: PROF_TAG=x BENCH_ARGS="--trunk sw --precision bf16" bash tools/prof_step.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-step}
mkdir -p $OUT
A="${BENCH_ARGS:-} --no-cpu-baseline --no-f32-exact --no-bf16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 2 $A > $OUT/bench_trace.json 2> $OUT/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 $A > /dev/null 2> $OUT/fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 $A > /dev/null 2> $OUT/write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o run -- python3 bench.py --steps 2 --warmup 1 $A > /dev/null 2> $OUT/mfma.err || exit $?
echo done
