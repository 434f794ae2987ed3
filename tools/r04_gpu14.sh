#!/bin/bash
# round 4, call 14: sparse counter with top-16-bit MSD passes + LDS chunk sort
# (k >= 9): parity suite, throughput vs the all-tile-pass path (KF_SPARSE_LSD=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r04/v14_pytest_sparse.log 2>&1 &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v14_sparse_bench.json 2> gpurun_out/r04/v14_sparse_bench.err &&
KF_SPARSE_LSD=1 timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v14_sparse_bench_lsd.json 2> gpurun_out/r04/v14_sparse_bench_lsd.err &&
timeout -k 10 400 python -u tools/r04_e2e_trace.py --parts 8:2,8:4,8:8,16:4,16:8,16:16,32:16 > gpurun_out/r04/v14_e2e_ahead.json 2> gpurun_out/r04/v14_e2e_ahead.err
