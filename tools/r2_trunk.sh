#!/bin/bash
# Whitening / IBN trunk evidence: per trunk (ibn, sw, isw; bf16, batch 16,
# 768x1024 -- the sta_* baseline configs) the bench line, a rocprofv3 kernel-trace summary,
# and PMC passes for HBM bytes (FETCH_SIZE, WRITE_SIZE) and MFMA-busy.  Optional 2nd arg
# "qnrf": the same for DensityRegressorBase fp16 at 2048x2048 (qnrf_final).
# Usage: PROF_TAG=r2t bash tools/r2_trunk.sh [ibn sw isw qnrf]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-r2t}
mkdir -p $OUT
LIST=${*:-ibn sw isw}
for T in $LIST; do
  if [ "$T" = qnrf ]; then
    A="--model DensityRegressorBase --mode simple --precision fp16 --height 2048 --width 2048 --batch 8 --no-bf16 --no-cpu-baseline"
  else
    A="--trunk $T --precision bf16 --no-bf16"
  fi
  D=$OUT/$T
  mkdir -p $D
  timeout -k 10 300 python3 bench.py $A --steps 5 --warmup 2 > $D/bench.json 2> $D/bench.err || { echo "bench $T failed"; tail -20 $D/bench.err; exit 1; }
  cat $D/bench.json
  P="$A --steps 1 --warmup 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A --steps 3 --warmup 1 > /dev/null 2> $D/trace.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py $P > /dev/null 2> $D/pmc1.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py $P > /dev/null 2> $D/pmc2.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 bench.py $P > /dev/null 2> $D/pmc3.err || exit $?
done
echo done
