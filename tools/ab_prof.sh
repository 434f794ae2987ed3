#!/bin/bash
# Phase profile (KF_BUCKET_PROFILE=1, s_memtime cycles per piece) of each library build.
#   LIBS="a.so b.so" K=11 bash tools/ab_prof.sh
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
for L in ${LIBS}; do
  KF_BUCKET_PROFILE=1 KF2VEC_GPU_LIB=$REPO/$L timeout -k 10 200 python3 "$REPO/tools/ab_bench.py" --variants 0 \
      --k ${K:-11} --rounds 1 --reps 2 > "$REPO/gpurun_out/ab_prof.log" 2>&1 || exit $?
  echo "$L"; grep -A16 "kf_bucket" "$REPO/gpurun_out/ab_prof.log" | tail -18
done
