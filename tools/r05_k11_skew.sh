#!/bin/bash
# k=11 bucket kernel against the record slots' placement (profiling build):
# physically contiguous scratch (KF_BUCKET_CONTIG=1) or not, and a hashed
# per-slot start skew of 0..63 x KF_BUCKET_SKEW bytes; one process per point.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05/k11skew}
mkdir -p "$OUT"
cd "$REPO"
export KF2VEC_GPU_LIB=$REPO/kf2vecfsw_amd/libkf2vec_gpu_ablation.so
POINTS=${POINTS:-"c:0 c:256 c:2048 c:16384 c:131072 n:0 n:2048 n:16384 n:0 n:2048 n:16384"}
for point in $POINTS; do
  mode=${point%%:*}; skew=${point#*:}
  if [ "$mode" = c ]; then export KF_BUCKET_CONTIG=1; else unset KF_BUCKET_CONTIG; fi
  KF_BUCKET_SKEW=$skew timeout -k 10 120 python3 -u tools/r04_run.py --k 11 --reps 10 > "$OUT/p.json" 2> "$OUT/p.err" \
    || { tail -5 "$OUT/p.err"; exit 1; }
  python3 -c "import json,statistics;x=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]);print(json.dumps({'contig':'$mode'=='c','skew_bytes':$skew,'median_ms':statistics.median(x['ms'][2:]),'ok':x['totals_analytic']}))" | tee -a "$OUT/skew.jsonl"
done
