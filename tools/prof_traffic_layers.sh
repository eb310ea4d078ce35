#!/bin/bash
# Per-launch HBM traffic of the fp32 headline's conv forward/dgrad launches against their
# algorithmic bytes: two PMC passes (FETCH_SIZE, WRITE_SIZE) of a 1-step bench with the launch
# list dumped (DGVCC_BENCH_LAUNCHES), joined by tools/traffic_layers.py.  Extra environment for
# the profiled runs: ENV="DGVCC_PSPLIT_ORDER=1" (A/B of the tile walk's traffic).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-tl}
mkdir -p $OUT
B="--no-cpu-baseline --no-bf16 --no-f32-exact --steps 1 --warmup 1"
env ${ENV:-} DGVCC_BENCH_LAUNCHES=$OUT/launches timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $B > $OUT/fetch.json 2> $OUT/fetch.err || exit $?
env ${ENV:-} timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $B > $OUT/write.json 2> $OUT/write.err || exit $?
echo done
