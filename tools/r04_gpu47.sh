#!/bin/bash
# sparse: re-order staged as 16-bit slot indices + key gather (sidx) vs keys staged (default)
set -e
mkdir -p gpurun_out/r04
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_sidx.so kf2vecfsw_amd/libkf2vec_gpu.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 13,16,21,31 --reps 5 > gpurun_out/r04/v47_$(basename $L .so).json
done
