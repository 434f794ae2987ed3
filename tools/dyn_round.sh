#!/bin/bash
# dynamic-chunk kernels: parity, A/B vs variant 1 and the pair kernel, lifetime profile
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-variants or pair or k7_kernel}" > "$OUT/pytest_dyn.log" 2>&1 || { tail -30 "$OUT/pytest_dyn.log"; exit 1; }
tail -1 "$OUT/pytest_dyn.log"
timeout -k 10 300 python -u tools/ab_bench.py --variants ${VARIANTS:-1,8,9,5} --k 7 --rounds 3 --reps 5 > "$OUT/ab_dyn.json" 2>> "$OUT/ab.err" || exit 1
python3 -c "import json;d=json.load(open('$OUT/ab_dyn.json'));print({k:round(v['median_ms'],4) for k,v in d['results'].items()})"
for v in ${PROF_VARIANTS:-8}; do
  KF_COUNT_PROFILE=1 KF_COUNT_VARIANT=$v timeout -k 10 120 python -u tools/ab_bench.py --variants $v --k 7 --rounds 1 --reps 2 > "$OUT/prof_v$v.log" 2>&1 || exit 1
  echo "variant $v"; grep -E "events|barrier-in|wave  0:|wave 15:" "$OUT/prof_v$v.log" | head -8
done
