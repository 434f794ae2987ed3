#!/bin/bash
# sparse u64 tile size re-measured on the single-sweep code: 4096 (default) vs 2048 vs 8192
set -e
mkdir -p gpurun_out/r04
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_t64_2048.so tools/ablib/libkf2vec_t64_8192.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 17,21,31 --reps 5 > gpurun_out/r04/v49_$(basename $L .so).json
done
