#!/bin/bash
# Parity subset for the given k=7 variants, then an in-process A/B (one GPU session).
#   VARIANTS=20,22 TESTS="-k 'variants_agree or u16 or many_pieces'" bash tools/ab_round.sh
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
V=${VARIANTS:-20,22}
if [ -n "${TESTS:-}" ]; then
  eval timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread $TESTS > "$OUT/pytest_ab.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_ab.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python tools/ab_bench.py --variants $V --rounds ${ROUNDS:-6} --reps 5 ${AB_ARGS:-} > "$OUT/ab.json" 2>&1 || exit $?
grep -E '^ "|median_ms|min_ms' "$OUT/ab.json"
