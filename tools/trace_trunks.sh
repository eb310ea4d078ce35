#!/bin/bash
# Kernel trace (no counters) of the three trunk steps, for per-launch grid / duration breakdowns
# (tools/grid_summary.py).  usage: PROF_TAG=x bash tools/trace_trunks.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-tt}
mkdir -p $OUT
for cfg in "isw:--trunk isw" "sw:--trunk sw --precision bf16" "ibn:--trunk ibn" "iswb:--trunk isw --precision bf16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 bench.py --steps 3 --warmup 2 $args --no-bf16 --no-cpu-baseline --no-f32-exact > $OUT/$name.json 2> $OUT/$name.err || exit $?
done
echo done
