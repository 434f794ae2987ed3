#!/bin/bash
# sparse: u32 tile 16384 (64-bit head masks) + u64 8192 (default) vs u32 8192; sparse tests first
set -e
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/v51_pytest_sparse.txt 2>&1
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_t32_8192.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 13,16,17,21,31 --reps 5 > gpurun_out/r04/v51_$(basename $L .so).json
done
