#!/bin/bash
# A/B of the f32 persistent conv (DGVCC_F32_PERSIST=1|0) on the headline workload, alternating in
# one call.  Usage: PROF_TAG=ab1 bash tools/ab_f32pers.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-ab}
mkdir -p $OUT
A="--no-bf16 --no-cpu-baseline --steps 4 --warmup 2"
for i in 1 2; do
  for f in 1 0; do
    DGVCC_F32_PERSIST=$f timeout -k 10 300 python3 bench.py $A > $OUT/bench_p${f}_$i.json 2> $OUT/bench_p${f}_$i.err || { echo "bench failed"; tail -5 $OUT/bench_p${f}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_p${f}_$i.json')); r=d['roofline']; print('persist=$f', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r['wgrad_frac'])"
  done
done
