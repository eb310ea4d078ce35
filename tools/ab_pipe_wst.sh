#!/bin/bash
# Same-box A/B of the 16-bit pipe kernel's 16-byte epilogue stores (DGVCC_PIPE_WST=0 vs default) on the
# bf16 final step and the SW bf16 trunk step, two alternations each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${PROF_TAG:-pipe_wst}; mkdir -p $OUT
for rep in 1 2; do
  for wst in 0 1; do
    for w in final sw; do
      extra=""; [ $w = sw ] && extra="--trunk sw"
      DGVCC_PIPE_WST=$wst timeout -k 10 200 python3 -u bench.py --precision bf16 --no-cpu-baseline --steps 10 --warmup 3 $extra > $OUT/${w}_wst${wst}_r$rep.json 2> $OUT/${w}_wst${wst}_r$rep.err || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'rep', sys.argv[4], d['value'], 'frames/s', d['ms_per_step'], 'ms')" $OUT/${w}_wst${wst}_r$rep.json $w wst=$wst $rep | tee -a $OUT/summary.txt
    done
  done
done
