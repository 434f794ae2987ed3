#!/bin/bash
# Bucket-kernel GPU tests, then in-process A/B (AB_K) of the current library against the
# previous bucket build (tools/ab/libkf2vec_fullwg.so) and the round-2 library.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_bucket.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_bucket.log"; [ $rc -eq 0 ] || exit $rc
for k in ${AB_K:-9 10 11 12}; do
timeout -k 10 300 python tools/lib_ab.py --libs ${AB_LIBS:-kf2vecfsw_amd/libkf2vec_gpu.so,tools/ab/libkf2vec_fullwg.so,tools/zoo/libkf2vec_zoo.so} --k $k --rounds 4 --reps 5 > "$OUT/lib_ab_k$k.json" 2>&1 || { echo "lib_ab rc=$?"; tail -5 "$OUT/lib_ab_k$k.json"; exit 1; }
python -c "
import json,sys
t=open('$OUT/lib_ab_k$k.json').read(); d=json.loads(t[t.index('{'):])
print('k=$k', d.get('counts_equal'), {p.split('/')[-1]:round(v['median_ms'],3) for p,v in d['results'].items()})"
done
