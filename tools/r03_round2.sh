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
