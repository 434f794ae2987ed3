#!/bin/bash
# Wave-slot balance experiments on K1x (variant 20): slot weights with the
# production library, and rotating s_setprio (libkf2vec_gpu_prio.so) with equal
# and slot weights; then per-wave profiles.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
run() {   # lib weights
  KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/$1 KF_WAVE_WEIGHTS=$2 timeout -k 10 150 python -u tools/ab_bench.py --variants ${VARIANT:-20} \
    --k 7 --rounds 4 --reps 5 > "$OUT/pr.json" 2> "$OUT/pr.err" || { tail -3 "$OUT/pr.err"; exit 1; }
  python3 -c "import json;t=open('$OUT/pr.json').read();d=json.loads(t[t.index('{'):]);print('$1 $2', {k:(round(v['median_ms'],4),round(v['min_ms'],4)) for k,v in d['results'].items()})"
}
for i in 1 2; do
  run libkf2vec_gpu.so 13,10,8,6
  run libkf2vec_gpu.so 16,11,8,5
  run libkf2vec_gpu.so 20,13,9,5
  run libkf2vec_gpu_prio.so 1,1,1,1
  run libkf2vec_gpu_prio.so 13,10,8,6
done
for L in libkf2vec_gpu.so:13,10,8,6 libkf2vec_gpu_prio.so:1,1,1,1; do
  KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/${L%%:*} KF_WAVE_WEIGHTS=${L##*:} KF_COUNT_PROFILE=1 timeout -k 10 120 python -u tools/ab_bench.py \
    --variants ${VARIANT:-20} --k 7 --rounds 1 --reps 1 > "$OUT/pr_prof.log" 2>&1 || exit 1
  echo "== $L"; grep -E "flushes|wave " "$OUT/pr_prof.log" | tail -17
done
