#!/bin/bash
# iteration check: conv kernel + model + trunk-kernel GPU tests, f32 conv A/B (fwd, wgrad), fp32 step
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-iter}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_trunk_kernels_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_f32conv.py 5 > $OUT/ab.txt 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
DGVCC_AB_KIND=wgrad timeout -k 10 300 python3 tools/ab_f32conv.py 5 > $OUT/ab_wgrad.txt 2> $OUT/ab_wgrad.err || { tail $OUT/ab_wgrad.err; exit 1; }
cat $OUT/ab.txt $OUT/ab_wgrad.txt
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-bf16 --no-f32-exact > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'fwd',r['achieved'],r['kernel_ms_per_step'],'wgrad',r['wgrad_achieved'],r['wgrad_ms_per_step'])"
