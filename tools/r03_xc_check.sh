#!/bin/bash
# GPU suite on the current library (k=7/8 coalesced layout), then the in-process A/B of
# k=7 and k=8 against the 48-byte-lane build (tools/ab/libkf2vec_x48.so).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_xc.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_xc.log"; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" "$OUT/pytest_xc.log" | head -60; exit $rc; }
for k in ${AB_K:-7 8}; do
timeout -k 10 300 python tools/lib_ab.py --libs ${AB_LIBS:-kf2vecfsw_amd/libkf2vec_gpu.so,tools/ab/libkf2vec_x48.so} --k $k --rounds 4 --reps 5 > "$OUT/lib_ab_xc_k$k.json" 2>&1 || { echo "lib_ab rc=$?"; tail -5 "$OUT/lib_ab_xc_k$k.json"; exit 1; }
python tools/ab_summary.py "$OUT/lib_ab_xc_k$k.json"
done
