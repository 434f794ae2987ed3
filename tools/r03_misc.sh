#!/bin/bash
# get_chunks windows/s, the new hand-off GPU test, and a 4-rank one-GPU rehearsal of the
# configs[3] mode on a resident 8,000-genome batch (2,000 genomes = 10 GB per rank)
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "features or chunk" > "$OUT/pytest_misc.log" 2>&1 || { echo "pytest rc=$?"; tail -20 "$OUT/pytest_misc.log"; exit 1; }
tail -1 "$OUT/pytest_misc.log"
timeout -k 10 400 python tools/chunks_bench.py --genomes 32 --reps 2 > "$OUT/chunks_bench.json" 2>"$OUT/chunks_bench.err" || { echo "chunks_bench rc=$?"; tail -5 "$OUT/chunks_bench.err"; exit 1; }
cat "$OUT/chunks_bench.json"
KF_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 3 --warmup 1 --total-genomes 8000 \
  > "$OUT/rehearse_configs3_4ranks_resident.log" 2>&1 || { echo "rehearse rc=$?"; tail -20 "$OUT/rehearse_configs3_4ranks_resident.log"; exit 1; }
grep '^{' "$OUT/rehearse_configs3_4ranks_resident.log" | cut -c1-600
