#!/bin/bash
# sparse scatter ablations (profiling only, wrong order by design): 1 no look-back, 2 no global stores, 3 no rank atomics
set -e
mkdir -p gpurun_out/r04
for L in kf2vecfsw_amd/libkf2vec_gpu.so tools/ablib/libkf2vec_sabl1.so tools/ablib/libkf2vec_sabl2.so tools/ablib/libkf2vec_sabl3.so; do
  echo "== $L" >&2
  KF2VEC_GPU_LIB=$PWD/$L timeout -k 10 240 python -u tools/sparse_bench.py --genomes 64 --k 16,31 --reps 4 > gpurun_out/r04/v37_$(basename $L .so).json
done
