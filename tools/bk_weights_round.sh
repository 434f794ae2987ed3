#!/bin/bash
# K3 phase-2 slot weights (KF_BK_WEIGHTS): parity suite under a skewed set, then
# k=11 kernel time per weight set, alternating, each in its own process.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
KF_BK_WEIGHTS=${PARITY_W:-3,2,2,1} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_bkw.log" 2>&1 || { tail -30 "$OUT/pytest_bkw.log"; exit 1; }
tail -1 "$OUT/pytest_bkw.log"
for i in $(seq 1 ${REPEAT:-2}); do
  for W in ${WSETS:-1,1,1,1 6,5,5,4 9,8,6,5 3,2,2,1}; do
    KF_BK_WEIGHTS=$W timeout -k 10 200 python3 tools/ab_bench.py --variants 1 --k 11 --rounds 2 --reps 5 \
      > "$OUT/bkw.json" 2> "$OUT/bkw.err" || { tail -5 "$OUT/bkw.err"; exit 1; }
    echo "$W $(grep -m1 median_ms "$OUT/bkw.json")"
  done
done
for W in 1,1,1,1 9,8,6,5; do
  KF_BUCKET_PROFILE=1 KF_BK_WEIGHTS=$W timeout -k 10 200 python3 tools/ab_bench.py --variants 1 --k 11 --rounds 1 --reps 1 \
    > /dev/null 2> "$OUT/bkw_prof_${W//,/}.err" || { tail -5 "$OUT/bkw_prof_${W//,/}.err"; exit 1; }
done
