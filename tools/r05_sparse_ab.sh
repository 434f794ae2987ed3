#!/bin/bash
# Sparse counter build variants, one process each, alternated twice:
#   LIBS="st8 sw8" bash tools/r05_sparse_ab.sh   (kf2vecfsw_amd/libkf2vec_gpu_<v>.so; "" = product)
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05/sparseab}
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2; do
  for v in "" ${LIBS}; do
    KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu${v:+_$v}.so timeout -k 10 200 python3 -u tools/sparse_bench.py \
      --genomes 64 --k 13,31 --reps 5 > "$OUT/p.json" 2> "$OUT/p.err" || { tail -5 "$OUT/p.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'${v:-product}','ms':{k:v['ms'] for k,v in d['k'].items()},'ok':[v['totals_ok'] for v in d['k'].values()]}))" | tee -a "$OUT/ab.jsonl"
  done
done
