#!/bin/bash
# k=11: what phase 2's barriers cost.  Processes alternated (one per library and
# repetition): the product, no barrier after each bucket's flush (ablation 10),
# no phase-2 barriers (11), phase 1 only (8).  Ablations count wrongly by design.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-r05/k11bar}
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2 3; do
  for v in "" abl10 abl11 abl8; do
    lib=$REPO/kf2vecfsw_amd/libkf2vec_gpu${v:+_$v}.so
    KF2VEC_GPU_LIB=$lib timeout -k 10 120 python3 -u tools/r04_run.py --k 11 --reps 10 > "$OUT/p.json" 2> "$OUT/p.err" \
      || { tail -5 "$OUT/p.err"; exit 1; }
    python3 -c "import json,statistics;x=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'${v:-product}','median_ms':statistics.median(x['ms'][2:])}))" | tee -a "$OUT/bar.jsonl"
  done
done
