#!/bin/bash
# emit: vector walk-back + half-row staging (default) vs serial walk-back + half rows (emit2) vs the round-4 emit (emit0)
set -e
mkdir -p gpurun_out/r04
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_emit0.so tools/ablib/libkf2vec_emit2.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 16,21,31 --reps 5 > gpurun_out/r04/v31_$(basename $L .so).json
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/v31_pytest_sparse.txt 2>&1
