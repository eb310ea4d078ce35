#!/bin/bash
# GPU check of the ResNet-trunk kernels and models (each step time-limited).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_trunk_kernels_gpu.py -q -x > gpurun_out/trunk_k.log 2>&1
rc=$?; echo "kernels rc=$rc" >> gpurun_out/trunk_k.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 500 python -m pytest tests/test_trunk_model_gpu.py -q > gpurun_out/trunk_m.log 2>&1
rc2=$?; echo "models rc=$rc2" >> gpurun_out/trunk_m.log
exit $(( rc > rc2 ? rc : rc2 ))
