#!/bin/bash
# round 4, call 9 (re-entry): full GPU suite on the pwrite row-writer tree, host
# formatter cost, traced get_chunks throughput, driver-args bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v9_pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u tools/fmt_bench.py --threads 16 > gpurun_out/r04/v9_fmt_bench.json 2>&1 &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 3 \
    > gpurun_out/r04/v9_chunks_bench.json 2> gpurun_out/r04/v9_chunks_bench.err &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v9_bench.json 2> gpurun_out/r04/v9_bench.err
