#!/bin/bash
# VALU issue table + SQ counters of K1 (variant 1) vs K1w (variant 13).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
timeout -k 10 120 "$REPO/tools/bin/valu_rate" > "$OUT/valu_rate.txt" 2>&1 || exit $?
tail -6 "$OUT/valu_rate.txt"
PMC_VARIANTS="${PMC_VARIANTS:-1 13}" bash "$REPO/tools/pmc_pair.sh"
