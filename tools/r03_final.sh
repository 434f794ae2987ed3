#!/bin/bash
# Round-3 evidence set: GPU suite, smoke, bench line, rocprofv3 kernel-trace stats of the
# bench command, HBM traffic passes (TRAFFIC_K, default "7 11").
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -f csv -- python3 "$REPO/bench.py" --steps 50 --warmup 10 --no-cpu --verify 0 > "$OUT/prof.log" 2>&1 || { echo "rocprof rc=$?"; tail -5 "$OUT/prof.log"; exit 1; }
tail -1 "$OUT/prof.log" | cut -c1-300
cd "$REPO"
K_LIST="${TRAFFIC_K:-7 11}" ROUND=r03 bash tools/traffic_round.sh || exit $?
