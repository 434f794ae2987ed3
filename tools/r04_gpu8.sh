#!/bin/bash
# round 4, call 8: get_chunks with the SSE2 row formatter and the block-streaming
# pwrite writer: chunk tests, host writer cost, traced throughput
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -k "chunk" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v8_pytest_chunks.log 2>&1 &&
timeout -k 10 120 python -u tools/fmt_bench.py --threads 16 > gpurun_out/r04/v8_fmt_bench.json 2>&1 &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 3 > gpurun_out/r04/v8_chunks_bench.json 2> gpurun_out/r04/v8_chunks_bench.err
