#!/bin/bash
# bench.py lines for K1 (variant 1) and the K1w variants, plus an in-process A/B.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
for v in ${BENCH_VARIANTS:-1 12 13}; do
  KF_COUNT_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --secondary-k 0 > "$OUT/bench_v$v.json" 2> "$OUT/bench_v$v.err" || exit $?
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_v$v.json')); print($v, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])"
done
timeout -k 10 300 python -u tools/ab_bench.py --variants ${AB_VARIANTS:-1,12,13} --k 7 --rounds 4 --reps 5 > "$OUT/wide_ab.json" 2> "$OUT/wide_ab.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/wide_ab.json'))['results']; [print(k, round(v['median_ms'],4), round(v['min_ms'],4)) for k,v in d.items()]"
