#!/bin/bash
# SQ counters of the k=7 kernels: variant 1 (forward histogram) vs 5 (pair).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
G=$'SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE\nSQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD'
for v in ${PMC_VARIANTS:-1 5}; do
  PAT=count_kernel; [ $v -ge 5 ] && PAT=pair_kernel; [ $v -ge 8 ] && PAT=dyn_kernel; [ $v -ge 10 ] && PAT=count_kernel
  PMC_TAG=pmc_v$v VARIANT=$v GROUPS_LIST="$G" bash "$REPO/tools/pmc_variant.sh" || exit $?
  cd "$REPO"
  python3 tools/pmc_summary.py gpurun_out/pmc_v$v $PAT > gpurun_out/pmc_v$v/summary.txt
  echo "== variant $v"; cat gpurun_out/pmc_v$v/summary.txt
done
