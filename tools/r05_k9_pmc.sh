#!/bin/bash
# PMC passes for k = 8 (K1x8), k = 9 (K1x9, tools/zoo/k1x9_two_part.patch applied)
# and the K1x9 variant that adds 0
# for the other part's windows (kf2vecfsw_amd/libk9_nomask.so).
#   tools/r05_k9_pmc.sh TAG
set -u
TAG=${1:-r05/k9pmc}
G=$'SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES\nSQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAVES'
K=8 TAG=$TAG/k8 GROUPS_LIST="$G" bash tools/r04_pmc.sh || exit 1
K=9 TAG=$TAG/k9 GROUPS_LIST="$G" bash tools/r04_pmc.sh || exit 1
LIB=kf2vecfsw_amd/libk9_nomask.so K=9 TAG=$TAG/k9nomask GROUPS_LIST="$G" bash tools/r04_pmc.sh || exit 1
