#!/bin/bash
# Variant 24 (k = 8 single pass on the K1x front end): parity, then A/B against K2 (variant 1 at k = 8).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "k8_single_pass" > "$OUT/pytest_k8.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_k8.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_bench.py --k 8 --variants 1,24 --rounds 4 --reps 5 > "$OUT/ab_k8.json" 2> "$OUT/ab_k8.err"
