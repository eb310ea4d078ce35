#!/bin/bash
# A/B an environment switch on the headline workload (fp32 final mode), alternating twice in one
# call.  Usage: PROF_TAG=ab2 VAR=DGVCC_EPI_STATS VALS="1 0" bash tools/ab_env.sh [bench args]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-ab}
mkdir -p $OUT
A="${*:---no-bf16 --no-cpu-baseline --steps 4 --warmup 2}"
for i in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 bench.py $A > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { echo "bench failed"; tail -5 $OUT/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$i.json')); r=d['roofline']; print('$VAR=$v', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r['wgrad_frac'])"
  done
done
