#!/bin/bash
# shader clock (s_memtime vs s_memrealtime) of the k=7 kernels under KF_COUNT_PROFILE
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
for v in ${VARIANTS:-1 5}; do
  KF_COUNT_PROFILE=1 KF_COUNT_VARIANT=$v timeout -k 10 120 python -u tools/ab_bench.py --variants $v --k 7 --rounds 1 --reps 2 > "$OUT/clk_v$v.log" 2>&1 || exit 1
  echo "variant $v"; grep -E "clock|barrier-in" "$OUT/clk_v$v.log" | head -4
done
timeout -k 10 300 python -u tools/ab_bench.py --variants 1,5 --k 7 --rounds 2 --reps 5 > "$OUT/ab_clk.json" 2>> "$OUT/ab.err" || exit 1
python3 -c "import json;d=json.load(open('$OUT/ab_clk.json'));print({k:round(v['median_ms'],4) for k,v in d['results'].items()})"
