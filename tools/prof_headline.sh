#!/bin/bash
# rocprofv3 passes over the fp32 headline step ONLY (no bf16 / f32-exact legs), so the per-launch
# HBM bytes and MFMA-busy of the split-math kernels are not averaged with other precisions:
# kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-headline}
mkdir -p $OUT
B="--no-cpu-baseline --no-bf16 --no-f32-exact ${BENCH_EXTRA:-}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 2 $B > $OUT/bench_trace.json 2> $OUT/trace.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 $B > $OUT/bench_fetch.json 2> $OUT/fetch.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 $B > $OUT/bench_write.json 2> $OUT/write.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o run -- python3 bench.py --steps 1 --warmup 1 $B > $OUT/bench_mfma.json 2> $OUT/mfma.err || exit $?
echo done
