#!/bin/bash
# Variant 22 (claimed tail units) on one box: its parity tests, then an
# in-process A/B against variant 20 over KF_DYN_FRAC / KF_DYN_UNIT settings.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "claimed_units or many_pieces or (agree and 22) or (low_complexity and 22)" > "$OUT/pytest_claim.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_claim.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_bench.py --variants ${VARIANTS:-20,22} --rounds ${ROUNDS:-4} --reps 5 \
  --env "${ENVSETS:-KF_DYN_FRAC=0.85,KF_DYN_UNIT=2;KF_DYN_FRAC=0.75,KF_DYN_UNIT=2;KF_DYN_FRAC=0.9,KF_DYN_UNIT=1;KF_DYN_FRAC=0.8,KF_DYN_UNIT=4}" \
  > "$OUT/ab_claim.json" 2> "$OUT/ab_claim.err"
rc=$?; cat "$OUT/ab_claim.json"; [ $rc = 0 ] || exit $rc
# per-wave timeline of workgroup 0 for variant 22 (loop ends should bunch up)
[ "${TIMELINE:-1}" = 1 ] || exit 0
timeout -k 10 120 env KF_COUNT_VARIANT=22 KF_COUNT_PROFILE=1 KF_COUNT_TIMELINE=1 python tools/ab_bench.py --variants 22 \
  --rounds 1 --reps 1 > "$OUT/timeline_v22.txt" 2>&1
