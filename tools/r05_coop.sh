#!/bin/bash
# k=11 cooperative bucket kernel (libkf2vec_gpu_coop.so, -DKF_BK_COOP_K=11):
# the k >= 9 parity tests through it, then processes alternated against the product.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05/coop}
mkdir -p "$OUT"
cd "$REPO"
LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu_coop.so
KF2VEC_GPU_LIB=$LIB timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "bucket or configs4 or count_matrix or dropin or smoke" > "$OUT/pytest_coop.log" 2>&1 || { tail -30 "$OUT/pytest_coop.log"; exit 1; }
tail -1 "$OUT/pytest_coop.log"
for rep in 1 2 3; do
  for v in "" coop; do
    KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu${v:+_$v}.so timeout -k 10 120 python3 -u tools/r04_run.py --k 11 --reps 10 \
      > "$OUT/p.json" 2> "$OUT/p.err" || { tail -5 "$OUT/p.err"; exit 1; }
    python3 -c "import json,statistics;x=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'${v:-product}','median_ms':statistics.median(x['ms'][2:]),'ok':x['totals_analytic']}))" | tee -a "$OUT/ab.jsonl"
  done
done
