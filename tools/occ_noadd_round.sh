#!/bin/bash
# K1 (variant 1) and K1d (variant 8) with and without the fast path's LDS adds
# (-DKF_K1_NOADD, wrong counts by design), K1d at two and at one workgroup per CU
# (KF_WGS_PER_CU; read once per process): how much does the front end lose at 16 waves/CU?
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
for i in 1 2; do
  for L in gpu gpu_noadd; do
    for W in 2 1; do
      KF_WGS_PER_CU=$W KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_$L.so timeout -k 10 200 python3 tools/ab_bench.py \
        --variants 1,8 --k 7 --rounds 3 --reps 5 > "$OUT/occ.json" 2> "$OUT/occ.err" || { tail -5 "$OUT/occ.err"; exit 1; }
      python3 -c "import json;t=open('$OUT/occ.json').read();d=json.loads(t[t.index('{'):]);print('$L wgs/cu(dyn)=$W',{k:round(v['median_ms'],4) for k,v in d['results'].items()})"
    done
  done
done
