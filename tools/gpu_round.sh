#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout/fault stops the script.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
stop_if_fatal() { rc=$1; what=$2; echo "$what rc=$rc" >> "$OUT/steps.log"; case $rc in 0|1) ;; *) echo "FATAL $what rc=$rc"; exit $rc;; esac; }
: > "$OUT/steps.log"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; stop_if_fatal $? pytest
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; stop_if_fatal $? smoke
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; stop_if_fatal $? bench
tail -1 "$OUT/bench.log"
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -f csv -- python3 "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu --verify 0 > "$OUT/prof.log" 2>&1; stop_if_fatal $? rocprof
  cd "$REPO"
  find "$OUT/prof" -name "*stats*" | head
fi
