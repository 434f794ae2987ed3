#!/bin/bash
# k=11 phase-2 record groups: two alternating groups of 4 windows (product) vs one
# group of 8 windows (KF_BK_DB=0); processes alternated, three repetitions.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05/k11db}
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2 3; do
  for v in "" db0; do
    KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu${v:+_$v}.so timeout -k 10 120 python3 -u tools/r04_run.py --k 11 --reps 10 \
      > "$OUT/p.json" 2> "$OUT/p.err" || { tail -5 "$OUT/p.err"; exit 1; }
    python3 -c "import json,statistics;x=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'${v:-product}','median_ms':statistics.median(x['ms'][2:]),'ok':x['totals_analytic']}))" | tee -a "$OUT/ab.jsonl"
  done
done
