#!/bin/bash
# SQ counter passes over the fp32 headline step (bench.py, fp32 leg only), restricted to the
# pre-split conv kernels, for the idle-cycle attribution of VERDICT r4 item 1
# (tools/sq_attrib.py turns the csvs into the table).  One rocprofv3 run per pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${PROF_TAG:-sq_headline}
mkdir -p $OUT
B="--steps 1 --warmup 1 --no-cpu-baseline --no-bf16 --no-f32-exact ${BENCH_EXTRA:-}"
RX="${SQ_REGEX:-conv_fwd_psplit|conv_fwd_rsplit|conv_wgrad_split}"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_WAVES"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_BUSY_CU_CYCLES"
P4="SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_IFETCH"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o run -- python3 bench.py $B > $OUT/bench_p$i.json 2> $OUT/p$i.err || exit $?
  echo "pass $i done"
done
echo done
