#!/bin/bash
# Process-level A/B of library builds (alternating), one variant:
#   LIBS="libkf2vec_gpu_base.so libkf2vec_gpu.so" VARIANT=20 REPEAT=3 bash tools/lib_ab.sh
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
for i in $(seq 1 ${REPEAT:-3}); do
  for L in ${LIBS}; do
    KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/$L timeout -k 10 150 python3 "$REPO/tools/ab_bench.py" --variants ${VARIANT:-20} \
        --k 7 --rounds 3 --reps 5 > "$OUT/lib_ab.json" 2> "$OUT/lib_ab.err" || { tail -3 "$OUT/lib_ab.err"; exit 1; }
    python3 -c "import json;t=open('$OUT/lib_ab.json').read();d=json.loads(t[t.index('{'):]);print('$L', {k:(round(v['median_ms'],4),round(v['min_ms'],4)) for k,v in d['results'].items()})"
  done
done
