#!/bin/bash
# Same-box A/B of one environment switch on a bench workload, interleaved rounds.
# usage: bash tools/ab_env.sh VAR "v0 v1 ..." ROUNDS OUTDIR [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
var=$1; vals=$2; rounds=$3; out=$4; shift 4
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do for v in $vals; do
  env "$var=$v" timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > "$out/r${r}_$v.json" 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$out/r${r}_$v.json').read().strip().splitlines()[-1]);print('$var=$v round $r', d['ms_per_step'], 'ms', d['value'], d['unit'])"
done; done
