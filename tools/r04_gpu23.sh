#!/bin/bash
# round 4, call 23: sparse tiles of 8192 u32 / 2048 u64 keys: parity suite and throughput (twice)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r04/v23_pytest_sparse.log 2>&1 &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v23_sparse_bench.json 2> gpurun_out/r04/v23_sparse_bench.err &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v23_sparse_bench_2.json 2> gpurun_out/r04/v23_sparse_bench_2.err
