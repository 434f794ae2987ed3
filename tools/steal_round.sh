#!/bin/bash
# Variant 23 (iteration claims + stealing): its parity tests, then an in-process A/B against 19.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "stealing or (many_pieces and 23) or (agree and 23) or (low_complexity and 23) or (adversarial and 23)" \
  > "$OUT/pytest_steal.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_steal.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_bench.py --variants ${VARIANTS:-19,23} --rounds ${ROUNDS:-6} --reps 5 \
  > "$OUT/ab_steal.json" 2> "$OUT/ab_steal.err"
