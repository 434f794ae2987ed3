#!/bin/bash
# Process-level A/B of pair-kernel builds (prefetch distance, stream-only ablations).
set -u
LIBS="kf2vecfsw_amd/libkf2vec_gpu.so kf2vecfsw_amd/libkf2vec_gpu_pf2.so kf2vecfsw_amd/libkf2vec_gpu_pf4.so kf2vecfsw_amd/libkf2vec_gpu_pf8.so kf2vecfsw_amd/libkf2vec_gpu_pabl3.so kf2vecfsw_amd/libkf2vec_gpu_pabl3pf4.so" VARIANT=${VARIANT:-5} REPEAT=2 bash tools/ab_libs.sh && LIBS="kf2vecfsw_amd/libkf2vec_gpu.so" VARIANT=1 REPEAT=1 bash tools/ab_libs.sh
