#!/bin/bash
# Where the static-range pair kernel (variant 10) loses against K1 (variant 1):
# K1 at 2 and 1 workgroups per CU with and without its adds (-DKF_K1_NOADD), and
# variant 10 with plain adds (-DKF_PAIR_ABL=1) and without pair adds (=2).  All
# ablation builds count wrong by design.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
run() {   # lib wgs variants
  KF_WGS_PER_CU=$2 KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_$1.so timeout -k 10 200 python3 tools/ab_bench.py \
    --variants $3 --k 7 --rounds 3 --reps 5 > "$OUT/k1sabl.json" 2> "$OUT/k1sabl.err" || { tail -5 "$OUT/k1sabl.err"; exit 1; }
  python3 -c "import json;t=open('$OUT/k1sabl.json').read();d=json.loads(t[t.index('{'):]);print('$1 wgs/cu<=$2',{k:round(v['median_ms'],4) for k,v in d['results'].items()})"
}
for i in 1 2; do
  run gpu 2 1,10
  run gpu 1 1
  run gpu_noadd 2 1
  run gpu_noadd 1 1
  run gpu_pabl1 2 10
  run gpu_pabl2 2 10
done
