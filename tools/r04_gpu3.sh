#!/bin/bash
# round 4, call 3: full GPU suite after the get_chunks rewrite + get_chunks throughput
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v3_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 3 > gpurun_out/r04/v3_chunks_bench.json 2> gpurun_out/r04/v3_chunks_bench.err
