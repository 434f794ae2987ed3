#!/bin/bash
# sparse: genome-interleaved tile order + look-back window 8 (default) vs no order vs order with window 4 / 1
set -e
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/v39_pytest_sparse.txt 2>&1
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_noorder.so tools/ablib/libkf2vec_lbw4.so tools/ablib/libkf2vec_lbw1.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 13,16,21,31 --reps 5 > gpurun_out/r04/v39_$(basename $L .so).json
done
