#!/bin/bash
# Full default bench line (fp32 split + f32_exact + bf16 legs + dmap + CPU baseline with the
# full-frame parity), per-launch dump of the fp32 leg and a rocprofv3 kernel-stats pass.
# Usage: PROF_TAG=r2d bash tools/r2_prof.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
if [ "${ONLY:-all}" != prof ]; then
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
fi
DGVCC_BENCH_LAUNCHES=$OUT/launches timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bf16 --no-f32-exact > $OUT/launch_run.json 2> $OUT/launch_run.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_fp32 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bf16 --no-f32-exact > $OUT/trace_fp32.json 2> $OUT/trace_fp32.err || exit $?
echo done
