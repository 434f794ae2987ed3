#!/bin/bash
# round 4, call 4: k >= 9 experiments -- u16 phase-2 halves A/B, bucket phase profile,
# SQ counters of the full kernel and of the phase-1-only ablation (k = 11)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
for k in 11 12 10; do
  timeout -k 10 200 python -u tools/lib_ab.py --libs tools/ab/libkf2vec_u16off.so,tools/ab/libkf2vec_new.so --k $k \
      --rounds 4 --reps 3 > gpurun_out/r04/v4_lib_ab_k${k}_u16.json 2> gpurun_out/r04/v4_lib_ab_k${k}_u16.err || exit $?
done &&
for lib in new u16off; do
  KF_BUCKET_PROFILE=1 KF2VEC_GPU_LIB=$GRAFT_REPO_ROOT/tools/ab/libkf2vec_prof.so timeout -k 10 120 python -u tools/r04_run.py --k 11 --reps 2 \
      > gpurun_out/r04/v4_bucket_profile_k11.txt 2>&1 || exit $?
  break
done &&
G1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVES"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY"
LIB=tools/ab/libkf2vec_new.so K=11 TAG=r04/v4_pmc_k11_full GROUPS_LIST="$G1"$'\n'"$G2" bash tools/r04_pmc.sh &&
LIB=tools/ab/libkf2vec_abl8.so K=11 TAG=r04/v4_pmc_k11_phase1 GROUPS_LIST="$G1"$'\n'"$G2" bash tools/r04_pmc.sh &&
python3 tools/pmc_summary.py gpurun_out/r04/v4_pmc_k11_full bucket_kernel > gpurun_out/r04/v4_pmc_k11_full.txt &&
python3 tools/pmc_summary.py gpurun_out/r04/v4_pmc_k11_phase1 bucket_kernel > gpurun_out/r04/v4_pmc_k11_phase1.txt &&
timeout -k 10 200 python -u tools/r04_e2e_trace.py --parts 2,4,8,16 > gpurun_out/r04/v4_e2e_trace.json 2> gpurun_out/r04/v4_e2e_trace.err &&
timeout -k 10 60 ./tools/bin/lds_ops > gpurun_out/r04/v4_lds_ops.txt 2>&1
