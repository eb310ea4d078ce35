#!/bin/bash
# SQ counters (wave-cycle breakdown, LDS bank conflicts, MFMA busy) of single conv layers
# (tools/prof_conv_one.py, fwd + wgrad) in f32 (split math) and bf16;
# usage: PROF_TAG=x [SQ_TESTS=1] bash tools/prof_sq_conv.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-sq}; mkdir -p $OUT
if [ "${SQ_TESTS:-0}" = "1" ]; then
  DGVCC_PROF_DT=f32 timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py -k "split or f32 or psplit or rsplit or tap3" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for DT in f32 bf16; do
for L in "96 128 512 512 3 32" "384 512 64 64 3 4"; do
  T=${DT}_$(echo $L | tr ' ' _)
  DGVCC_PROF_DT=$DT timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$T -o run -- python3 tools/prof_conv_one.py $L fwd,wgrad > $OUT/t_$T.log 2>&1 || exit 1
  DGVCC_PROF_DT=$DT timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p_$T -o run -- python3 tools/prof_conv_one.py $L fwd,wgrad > $OUT/p_$T.log 2>&1 || exit 1
done
done
echo ok
