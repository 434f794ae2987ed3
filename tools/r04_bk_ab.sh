#!/bin/bash
# Bucket-kernel iteration: k>=9 GPU parity tests, then one-process A/B of the
# working-tree library against tools/ab/libkf2vec_head.so for K_LIST.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
TAG=${TAG:-bk}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$OUT/${TAG}_pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ALT_LIB:-}" ]; then   # the bucket-kernel GPU tests on an alternative build
  KF2VEC_GPU_LIB=$REPO/$ALT_LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "bucket or all_k or ragged or arbitrary or deterministic or unaligned or split or many_small or synth or fastq or short_lines" \
    > "$OUT/${TAG}_pytest_alt.log" 2>&1
  rc=$?; tail -2 "$OUT/${TAG}_pytest_alt.log"; [ $rc -eq 0 ] || exit $rc
fi
for k in ${K_LIST:-11 9 10 12}; do
  timeout -k 10 200 python3 tools/lib_ab.py --libs tools/ab/libkf2vec_head.so,kf2vecfsw_amd/libkf2vec_gpu.so${EXTRA_LIBS:-} \
     --k $k --rounds ${ROUNDS:-4} --reps 5 > "$OUT/${TAG}_ab_k$k.json" 2> "$OUT/${TAG}_ab_k$k.err" || { echo "ab k=$k rc=$?"; tail -5 "$OUT/${TAG}_ab_k$k.err"; exit 1; }
  python3 -c "import json;t=open('$OUT/${TAG}_ab_k$k.json').read();d=json.loads(t[t.index('{'):]);print('k=$k', d.get('counts_equal'), {k.split('/')[-1]:(round(v['median_ms'],3),round(v['min_ms'],3)) for k,v in d['results'].items()})"
done
