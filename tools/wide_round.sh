#!/bin/bash
# K1w round: parity of the wide-lane pair variants, then an in-process A/B
# against K1 (variant 1) and K1s (variant 10) on the bench batch.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "variants_agree or u16_drains" > "$OUT/wide_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/wide_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_bench.py --variants ${AB_VARIANTS:-1,10,12,13} --k 7 --rounds 4 --reps 5 \
  > "$OUT/wide_ab.json" 2> "$OUT/wide_ab.err"
rc=$?; cat "$OUT/wide_ab.json"; exit $rc
