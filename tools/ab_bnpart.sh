#!/bin/bash
# same-box A/B of DGVCC_DGRAD_BNPART on the bf16 final step
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab_bnpart
for r in 1 2; do for v in 0 1; do
  DGVCC_DGRAD_BNPART=$v timeout -k 10 150 python -u bench.py --precision bf16 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bnpart/r${r}_v$v.json 2>&1 || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_bnpart/r${r}_v$v.json').read().strip().splitlines()[-1]);print('bnpart=$v round $r', d['ms_per_step'])"
done; done
