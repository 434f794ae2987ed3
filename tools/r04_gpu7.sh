#!/bin/bash
# round 4, call 7: full GPU suite with weighted phase-2 rounds as the default and the
# concurrent get_chunks writer; traced get_chunks throughput; driver-args bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v7_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 3 \
    > gpurun_out/r04/v7_chunks_bench.json 2> gpurun_out/r04/v7_chunks_bench.err &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v7_bench.json 2> gpurun_out/r04/v7_bench.err
