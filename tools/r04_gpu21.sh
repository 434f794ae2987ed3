#!/bin/bash
# round 4, call 21: sparse counter with LDS-atomic ranks in the scatter (+ the device
# order check) and offset validation: parity suite; throughput vs ballot ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r04/v21_pytest_sparse.log 2>&1 &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v21_sparse_bench.json 2> gpurun_out/r04/v21_sparse_bench.err &&
KF2VEC_GPU_LIB=$GRAFT_REPO_ROOT/tools/ablib/libkf2vec_ballot.so timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v21_sparse_bench_ballot.json 2> gpurun_out/r04/v21_sparse_bench_ballot.err &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v21_sparse_bench_2.json 2> gpurun_out/r04/v21_sparse_bench_2.err
