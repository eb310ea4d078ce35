#!/bin/bash
# f32 conv A/B timing (forward and wgrad) + an SQ counter pass on one layer.
# Usage: PROF_TAG=ab2 PMC_KIND=wgrad bash tools/r2_ab.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-ab}
mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_f32conv.py 5 > $OUT/ab.txt 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
DGVCC_AB_KIND=wgrad timeout -k 10 300 python3 tools/ab_f32conv.py 5 > $OUT/ab_wgrad.txt 2> $OUT/ab_wgrad.err || { tail $OUT/ab_wgrad.err; exit 1; }
cat $OUT/ab.txt $OUT/ab_wgrad.txt
export DGVCC_AB_SHAPES="192,256,256,256,16"
DGVCC_AB_KIND=${PMC_KIND:-fwd} timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 tools/ab_f32conv.py 2 > /dev/null 2> $OUT/pmc.err || { tail -5 $OUT/pmc.err; exit 1; }
echo done
