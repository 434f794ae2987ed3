#!/bin/bash
# Lean product library: GPU parity suite, smoke, bench, rocprof stats, then
# in-process A/B against the round-2 zoo library at k=7 and k=11.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
SKIP_PROF=${SKIP_PROF:-0} bash tools/gpu_round.sh || exit $?
for k in 11 7; do
  timeout -k 10 300 python tools/lib_ab.py --libs kf2vecfsw_amd/libkf2vec_gpu.so,tools/zoo/libkf2vec_zoo.so --k $k \
    --rounds 4 --reps 5 > "$OUT/lib_ab_k$k.json" 2>&1 || { echo "lib_ab k=$k rc=$?"; tail -5 "$OUT/lib_ab_k$k.json"; exit 1; }
  grep -A3 median "$OUT/lib_ab_k$k.json" | head -12
done
timeout -k 10 400 python tools/chunks_bench.py --genomes 32 --reps 2 > "$OUT/chunks_bench.json" 2>"$OUT/chunks_bench.err" || { echo "chunks_bench rc=$?"; tail -5 "$OUT/chunks_bench.err"; exit 1; }
cat "$OUT/chunks_bench.json"
KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu_ablation.so KF_BUCKET_PROFILE=1 timeout -k 10 200 python tools/ab_bench.py --variants 19 --k 11 --rounds 1 --reps 2 > "$OUT/bk_prof_k11_r03.log" 2>&1 || exit 1
grep "pieces\|median" "$OUT/bk_prof_k11_r03.log" | head -4
