#!/bin/bash
# Bucket-kernel phase profile (profiling build, KF_BUCKET_PROFILE=1) for K_LIST.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
TAG=${TAG:-bk}
for k in ${PROF_K:-11}; do
  KF2VEC_GPU_LIB=$REPO/${PROF_LIB:-kf2vecfsw_amd/libkf2vec_gpu_ablation.so} KF_BUCKET_PROFILE=1 timeout -k 10 200 \
    python3 tools/lib_ab.py --libs ${PROF_LIB:-kf2vecfsw_amd/libkf2vec_gpu_ablation.so} --k $k --rounds 1 --reps 2 > "$OUT/${TAG}_prof_k$k.log" 2>&1 || { echo "prof k=$k rc=$?"; tail -5 "$OUT/${TAG}_prof_k$k.log"; exit 1; }
  grep -B1 -A17 "pieces" "$OUT/${TAG}_prof_k$k.log" | tail -19
done
