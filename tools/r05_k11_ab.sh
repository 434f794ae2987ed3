#!/bin/bash
# Round 5, k=11 phase-1 staging: in-process A/B of the product library against
# KF_BK_SWZ=1 (swizzled staging slots), KF_BK_RL11=1 (two rank replicas) and the
# no-staging-writes ablation (KF_BK_ABL=4, wrong counts: its own process), then
# phase-1-only LDS counters (KF_BK_ABL=8 builds) with and without the swizzle.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05/k11ab}
mkdir -p "$OUT"
cd "$REPO"
L=kf2vecfsw_amd
timeout -k 10 240 python3 -u tools/lib_ab.py --libs $L/libkf2vec_gpu.so,$L/libkf2vec_gpu_swz.so,$L/libkf2vec_gpu_rl1.so \
  --k 11 --rounds 4 --reps 5 > "$OUT/ab_k11.json" 2> "$OUT/ab_k11.err" || { tail -5 "$OUT/ab_k11.err"; exit 1; }
timeout -k 10 240 python3 -u tools/lib_ab.py --libs $L/libkf2vec_gpu.so,$L/libkf2vec_gpu_abl4.so \
  --k 11 --rounds 4 --reps 5 > "$OUT/ab_k11_abl4.json" 2> "$OUT/ab_k11_abl4.err"
rc=$?; [ $rc = 0 ] || [ $rc = 3 ] || { tail -5 "$OUT/ab_k11_abl4.err"; exit 1; }
for k in 12 10 9; do
  timeout -k 10 240 python3 -u tools/lib_ab.py --libs $L/libkf2vec_gpu.so,$L/libkf2vec_gpu_swz.so \
    --k $k --rounds 4 --reps 5 > "$OUT/ab_k$k.json" 2> "$OUT/ab_k$k.err" || { tail -5 "$OUT/ab_k$k.err"; exit 1; }
done
for v in abl8 abl8swz; do
  LIB=$L/libkf2vec_gpu_$v.so K=11 TAG=${TAG:-r05/k11ab}/pmc_$v \
    GROUPS_LIST="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
    bash tools/r04_pmc.sh || exit 1
done
echo done
