#!/bin/bash
# round 4: 2-rank one-GPU rehearsal of the multi-GPU bench path on the final tree
# (KF_BENCH_REHEARSE=1: both ranks on cuda:0 over gloo, each capped at 70 GB resident so two
# fit on one card; the driver's N>1 runs use RCCL, one GPU per rank)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
KF_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --max-resident-gb 70 \
  > gpurun_out/r04/v48_rehearse_2ranks.log 2>&1
