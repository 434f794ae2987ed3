#!/bin/bash
# sparse: branch-free base codes and window steps in the emit (default) vs the previous commit (prev); sparse tests first
set -e
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/v54_pytest_sparse.txt 2>&1
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_prev.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 13,16,17,21,31 --reps 5 > gpurun_out/r04/v54_$(basename $L .so).json
done
