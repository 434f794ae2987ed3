#!/bin/bash
# GPU suite on the current library, then in-process A/B (AB_K, default k=11) of the current
# library, the pre-half-workgroup bucket build (tools/ab) and the round-2 library (tools/zoo).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for k in ${AB_K:-11}; do
timeout -k 10 300 python tools/lib_ab.py --libs ${AB_LIBS:-kf2vecfsw_amd/libkf2vec_gpu.so,tools/ab/libkf2vec_fullwg.so,tools/zoo/libkf2vec_zoo.so} --k $k --rounds 4 --reps 5 > "$OUT/lib_ab_k$k.json" 2>&1 || { echo "lib_ab rc=$?"; tail -5 "$OUT/lib_ab_k$k.json"; exit 1; }
grep -A1 '\.so' "$OUT/lib_ab_k$k.json"
done
