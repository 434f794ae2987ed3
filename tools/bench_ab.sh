#!/bin/bash
# bench.py's own k=7 line under two kernel variants, alternating
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
for i in 1 2; do
  for v in ${VARIANTS:-1 5}; do
    KF_COUNT_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu --secondary-k 0 --verify 2 > "$OUT/bench_v$v.log" 2>> "$OUT/bench_ab.err" || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/bench_v$v.log').read().strip().splitlines()[-1]);print('variant $v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])"
  done
done
