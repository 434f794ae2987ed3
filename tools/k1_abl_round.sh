#!/bin/bash
# K1 ablations (python -m kf2vecfsw_amd.build --ablation; wrong counts by design):
# variant 3 = no LDS adds, 4 = stream only, against variant 1 in the same process
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
KF2VEC_GPU_LIB=${GRAFT_REPO_ROOT:-$(pwd)}/kf2vecfsw_amd/libkf2vec_gpu_ablation.so \
  timeout -k 10 300 python tools/ab_bench.py --variants 1,3,4 --k 7 --rounds 3 --reps 5 \
  > "$OUT/abl_k1.json" 2> "$OUT/abl_k1.err" || { tail -5 "$OUT/abl_k1.err"; exit 1; }
# (ab_bench prints "COUNTS DIFFER" lines before its JSON for these wrong-count builds)
python3 -c "import json;t=open('$OUT/abl_k1.json').read();d=json.loads(t[t.index('{'):]);print({k:round(v['median_ms'],4) for k,v in d['results'].items()})"
