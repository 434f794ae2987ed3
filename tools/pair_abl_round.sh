#!/bin/bash
# pair kernel ablations (wrong counts by design): 1 = plain ds_add (no returns/checks),
# 2 = no pair adds, 3 = stream only; against the real build, same box
set -u
LIBS="kf2vecfsw_amd/libkf2vec_gpu.so kf2vecfsw_amd/libkf2vec_gpu_pabl1.so kf2vecfsw_amd/libkf2vec_gpu_pabl2.so kf2vecfsw_amd/libkf2vec_gpu_pabl3.so" VARIANT=5 REPEAT=2 bash tools/ab_libs.sh
