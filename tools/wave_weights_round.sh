#!/bin/bash
# K1x wave-slot weights (KF_WAVE_WEIGHTS) sweep: one ab_bench process per set, then
# the per-wave profile of the last set.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
for W in ${WSETS:-1,1,1,1 9,8,7,6 11,9,7,6 13,10,8,6 16,12,9,7 1,1,1,1}; do
  KF_WAVE_WEIGHTS=$W timeout -k 10 120 python -u tools/ab_bench.py --variants ${VARIANT:-18} --k 7 --rounds 3 --reps 5 \
    > "$OUT/ww.json" 2> "$OUT/ww.err" || { tail -3 "$OUT/ww.err"; exit 1; }
  python3 -c "import json;t=open('$OUT/ww.json').read();d=json.loads(t[t.index('{'):]);print('$W', {k:(round(v['median_ms'],4),round(v['min_ms'],4)) for k,v in d['results'].items()})"
done
KF_WAVE_WEIGHTS=${PROF_W:-13,10,8,6} KF_COUNT_PROFILE=1 timeout -k 10 120 python -u tools/ab_bench.py --variants ${VARIANT:-18} --k 7 --rounds 1 --reps 1 > "$OUT/ww_prof.log" 2>&1 || exit 1
grep -E "clock|kernel|wave " "$OUT/ww_prof.log" | head -22
