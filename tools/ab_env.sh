#!/bin/bash
# Same-box A/B of env switches: AB_VARS="DGVCC_X=0 DGVCC_X=1 ..." -> one bench line each.
set -u
mkdir -p gpurun_out/ab_env
for v in ${AB_VARS}; do
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/ab_env/$v.json 2> gpurun_out/ab_env/$v.err || { echo "$v failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], 'conv', r['achieved'], r['kernel_ms_per_step'], 'wgrad', r['wgrad_achieved'], r['wgrad_ms_per_step'])" gpurun_out/ab_env/$v.json $v
done
