#!/bin/bash
# SQ counters of K1w (variant 13) vs K1x (variant 18), plus an instruction-fetch pass.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
G=$'SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE\nSQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD\nSQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES'
for v in ${PMC_VARIANTS:-13 18}; do
  PMC_TAG=pmc_v$v VARIANT=$v GROUPS_LIST="$G" bash "$REPO/tools/pmc_variant.sh" || exit $?
  cd "$REPO"
  python3 tools/pmc_summary.py gpurun_out/pmc_v$v count_kernel > gpurun_out/pmc_v$v/summary.txt
  echo "== variant $v"; cat gpurun_out/pmc_v$v/summary.txt
done
