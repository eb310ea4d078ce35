#!/bin/bash
# Secondary workloads on the current build (one box): final mode at 768x1024 and at the shipped
# 320-px crops, the three ResNet trunks, and eval.  Each run has its own time limit.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sweep_r1i
mkdir -p $OUT
B="timeout -k 10 240 python bench.py --no-cpu-baseline"
$B --mode final --steps 8 --warmup 3 > $OUT/s_final.json || exit $?
$B --mode final --height 320 --width 320 --steps 20 --warmup 5 > $OUT/s_final320.json || exit $?
for t in sw isw ibn; do $B --trunk $t --steps 8 --warmup 3 > $OUT/s_trunk_$t.json || exit $?; done
timeout -k 10 240 python tools/bench_eval.py > $OUT/s_eval.json 2> $OUT/s_eval.err || exit $?
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d.get('value'), d.get('unit'), d.get('ms_per_step'))" $f; done
