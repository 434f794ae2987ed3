#!/bin/bash
# Does pair counting pay at two workgroups per CU?  pabl1 = plain-add pairs, one
# workgroup/CU (128 KiB P); pabl4 = same adds into a 64 KiB P, two workgroups/CU
# (wrong counts by design, both); variant 1 = K1 in the same process.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
for L in pabl1 pabl4; do
  KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu_$L.so timeout -k 10 300 python3 tools/ab_bench.py \
    --variants 1,6,5 --k 7 --rounds 3 --reps 5 > "$OUT/half_$L.json" 2> "$OUT/half_$L.err" \
    || { tail -5 "$OUT/half_$L.err"; exit 1; }
  python3 -c "import json;t=open('$OUT/half_$L.json').read();d=json.loads(t[t.index('{'):]);print('$L',{k:round(v['median_ms'],4) for k,v in d['results'].items()})"
done
