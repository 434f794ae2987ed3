#!/bin/bash
# Wave-priority A/B of the bucket kernel (KF_BK_PRIO builds), then rocprofv3
# kernel-trace stats of the bench at its default warmup / steps.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
TESTS=0 TAG=v22 K_LIST="11 10 12 9" EXTRA_LIBS=",tools/ab/libkf2vec_prio1.so,tools/ab/libkf2vec_prio2.so,tools/ab/libkf2vec_prio3.so" \
  bash tools/r04_bk_ab.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -f csv -- python3 "$REPO/bench.py" --steps 50 --warmup 10 --no-cpu --verify 0 > "$OUT/prof.log" 2>&1 || { echo "rocprof rc=$?"; tail -5 "$OUT/prof.log"; exit 1; }
tail -1 "$OUT/prof.log" | cut -c1-300
