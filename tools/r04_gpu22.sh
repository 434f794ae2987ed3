#!/bin/bash
# round 4, call 22: sparse counter with 8192-key tiles (dynamic LDS staging): parity suite;
# throughput vs 2048-key tiles (same sources, -DKF_SPARSE_TILE=2048)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r04/v22_pytest_sparse.log 2>&1 &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v22_sparse_bench.json 2> gpurun_out/r04/v22_sparse_bench.err &&
KF2VEC_GPU_LIB=$GRAFT_REPO_ROOT/tools/ablib/libkf2vec_t2048.so timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v22_sparse_bench_t2048.json 2> gpurun_out/r04/v22_sparse_bench_t2048.err &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v22_sparse_bench_2.json 2> gpurun_out/r04/v22_sparse_bench_2.err
