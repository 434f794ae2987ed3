#!/bin/bash
# Marginal cost of VALU work inside K1x: the production library against builds
# with 48 extra VALU ops per 3 KiB iteration (tools/build_abl.sh -DKF_K1X_PAD=...).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
for i in 1 2; do
  for L in ${PAD_LIBS:-libkf2vec_gpu.so libkf2vec_gpu_pad1.so libkf2vec_gpu_pad2.so libkf2vec_gpu_pad3.so libkf2vec_gpu_pad4.so}; do
    KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/$L timeout -k 10 200 python3 "$REPO/tools/ab_bench.py" --variants ${VARIANT:-18} --k 7 \
        --rounds 3 --reps 5 > "$OUT/pad.log" 2>&1 || { tail -5 "$OUT/pad.log"; exit 1; }
    python3 -c "import json;t=open('$OUT/pad.log').read();d=json.loads(t[t.index('{'):]);print('$L', {k:(round(v['median_ms'],4),round(v['min_ms'],4)) for k,v in d['results'].items()})"
  done
done
