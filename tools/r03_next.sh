#!/bin/bash
# Bucket check (GPU suite + A/B), the LDS rank microbenchmark, then r03_misc.sh.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
bash tools/r03_bucket_check.sh || exit $?
timeout -k 10 120 tools/ab/lds_rank > "$OUT/lds_rank.txt" 2>&1 || { echo "lds_rank rc=$?"; tail -5 "$OUT/lds_rank.txt"; exit 1; }
cat "$OUT/lds_rank.txt"
bash tools/r03_misc.sh
