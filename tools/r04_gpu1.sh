#!/bin/bash
# round 4, call 1: cold-launch diagnosis + the driver's bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 240 python -u tools/r04_cold.py > gpurun_out/r04/v1_cold.json 2> gpurun_out/r04/v1_cold.err &&
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v1_bench.json 2> gpurun_out/r04/v1_bench.err
