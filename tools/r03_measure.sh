#!/bin/bash
# bench line + in-process A/B vs the round-2 library (zoo) + bucket phase profile
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
for k in ${AB_K:-11 7}; do
  timeout -k 10 300 python tools/lib_ab.py --libs kf2vecfsw_amd/libkf2vec_gpu.so,tools/zoo/libkf2vec_zoo.so --k $k \
    --rounds 4 --reps 5 > "$OUT/lib_ab_k$k.json" 2>&1 || { echo "lib_ab k=$k rc=$?"; tail -5 "$OUT/lib_ab_k$k.json"; exit 1; }
  grep -B1 -A2 median "$OUT/lib_ab_k$k.json" | head -12
done
KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu_ablation.so KF_BUCKET_PROFILE=1 timeout -k 10 200 python tools/ab_bench.py --variants 19 --k 11 --rounds 1 --reps 2 > "$OUT/bk_prof_k11_r03.log" 2>&1 || exit 1
grep "pieces" "$OUT/bk_prof_k11_r03.log" | head -2
