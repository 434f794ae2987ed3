#!/bin/bash
# Round 5, k=11: (1) position bias of the in-process A/B (tools/lib_ab.py) with
# four copies of ONE library (each copy has its own workspace allocation);
# (2) process-level alternation (one process per library and repetition, the
# same allocation order in each) of R = 1, R = 2, W = 8 (R = 1, 2) and equal
# phase-2 round weights.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05/k11ab3}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
L=kf2vecfsw_amd
timeout -k 10 300 python3 -u tools/lib_ab.py --libs $L/libkf2vec_gpu_rl0.so,$L/libkf2vec_gpu_rl0_c1.so,$L/libkf2vec_gpu_rl0_c2.so,$L/libkf2vec_gpu_rl0_c3.so \
  --k 11 --rounds 4 --reps 5 > "$OUT/bias_k11.json" 2> "$OUT/bias_k11.err" || { tail -5 "$OUT/bias_k11.err"; exit 1; }
for rep in 1 2 3; do
  for v in rl0 "" w8 w8r2 rw0; do
    lib=$L/libkf2vec_gpu${v:+_$v}.so
    KF2VEC_GPU_LIB=$REPO/$lib timeout -k 10 120 python3 -u tools/r04_run.py --k 11 --reps 12 >> "$OUT/proc_k11.jsonl" 2>> "$OUT/proc_k11.err" \
      || { tail -5 "$OUT/proc_k11.err"; exit 1; }
  done
done
echo done
