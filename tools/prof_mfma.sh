#!/bin/bash
# rocprofv3 PMC pass for MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs)
# and GRBM_GUI_ACTIVE (summed over the 8 XCDs) per dispatch of one bench step.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-mfma}
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-} > $OUT/bench_mfma.json 2> $OUT/mfma.err || exit $?
echo done
