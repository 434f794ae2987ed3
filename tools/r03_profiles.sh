#!/bin/bash
# Round-3 evidence: rocprofv3 kernel-trace stats of the bench command, HBM
# traffic PMC passes (k=7, 8, 11), the GPU suite log and smoke.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -f csv -- python3 "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu --verify 0 > "$OUT/prof.log" 2>&1 || { echo "rocprof rc=$?"; tail -5 "$OUT/prof.log"; exit 1; }
tail -1 "$OUT/prof.log"
find "$OUT/prof" -name "*kernel_stats*"
cd "$REPO"
K_LIST="7 8 11" ROUND=r03 bash tools/traffic_round.sh || exit $?
cat "$OUT"/traffic_k*.json
