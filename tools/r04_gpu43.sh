#!/bin/bash
# sparse: persistent single-sweep passes with next-tile prefetch (default) vs one tile per workgroup (nopersist) vs non-temporal (nt, one tile per workgroup); sparse tests first
set -e
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/v43_pytest_sparse.txt 2>&1
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_nopersist.so tools/ablib/libkf2vec_nt.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 13,16,21,31 --reps 5 > gpurun_out/r04/v43_$(basename $L .so).json
done
