#!/bin/bash
# K1w ablations (tools/build_abl.sh -DKF_K1W_ABL=N; wrong counts by design):
# the production library and each ablation library, alternating, variant 13.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
for i in 1 2; do
  for L in libkf2vec_gpu.so libkf2vec_gpu_k1wabl1.so libkf2vec_gpu_k1wabl2.so libkf2vec_gpu_k1wabl4.so; do
    KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/$L timeout -k 10 200 python3 "$REPO/tools/ab_bench.py" --variants ${VARIANT:-13} --k 7 \
        --rounds 3 --reps 5 > "$OUT/k1w_abl.log" 2>&1 || { tail -5 "$OUT/k1w_abl.log"; exit 1; }
    python3 -c "import json;t=open('$OUT/k1w_abl.log').read();d=json.loads(t[t.index('{'):]);print('$L', {k:(round(v['median_ms'],4),round(v['min_ms'],4)) for k,v in d['results'].items()})"
  done
done
