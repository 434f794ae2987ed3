#!/bin/bash
# Process-level A/B of two library builds on one GPU box, alternating runs.
#   LIBS="a.so b.so" K=7 REPEAT=3 VARIANT=2 bash tools/ab_libs.sh
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
for i in $(seq 1 ${REPEAT:-3}); do
  for L in ${LIBS}; do
    KF2VEC_GPU_LIB=$REPO/$L timeout -k 10 200 python3 "$REPO/tools/ab_bench.py" --variants ${VARIANT:-2} --k ${K:-7} \
        --rounds 2 --reps 5 > "$REPO/gpurun_out/ab_lib.log" 2>&1 || exit $?
    echo "$L $(grep -m1 median_ms "$REPO/gpurun_out/ab_lib.log")"
  done
done
