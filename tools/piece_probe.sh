#!/bin/bash
# Per-piece cost probe (K1x): flush sub-phase timeline of workgroup 0 and the
# genome-size sweep (same bytes in 250 / 1000 / 4000 genomes).  One GPU session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
V=${VARIANTS:-20}
timeout -k 10 120 env KF_COUNT_PROFILE=1 KF_COUNT_TIMELINE=1 python tools/ab_bench.py --variants ${V%%,*} --rounds 1 --reps 1 > "$OUT/timeline.txt" 2>&1 || exit $?
for gs in "250 20000000" "1000 5000000" "4000 1250000"; do
  set -- $gs
  echo "== genomes $1 x $2" >> "$OUT/sweep.txt"
  timeout -k 10 180 python tools/ab_bench.py --variants $V --rounds 3 --reps 5 --genomes $1 --seq-len $2 >> "$OUT/sweep.txt" 2>&1 || exit $?
done
