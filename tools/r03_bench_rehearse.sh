#!/bin/bash
# Round 3: default bench line (configs[1], all-core CPU baseline) and a 2-rank
# one-GPU rehearsal of the configs[3] 50k-genome mode (streamed sub-batches).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
KF_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --max-resident-gb 70 \
  > "$OUT/rehearse_50k_2ranks.log" 2>&1 || { echo "rehearse rc=$?"; tail -20 "$OUT/rehearse_50k_2ranks.log"; exit 1; }
tail -1 "$OUT/rehearse_50k_2ranks.log"
if [ "${BK_PROF:-1}" = 1 ]; then
  KF_BUCKET_PROFILE=1 timeout -k 10 200 python tools/ab_bench.py --variants 19 --k 11 --rounds 1 --reps 2 > "$OUT/bk_prof_k11.log" 2>&1 || exit 1
  grep -v "^ *$" "$OUT/bk_prof_k11.log" | head -30
fi
