#!/bin/bash
# parity suite on the working tree, then process-level A/B of the working tree's
# library against kf2vecfsw_amd/libkf2vec_gpu_prev.so (tools/build_rev.sh)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_lib_ab.log" 2>&1 || { tail -30 "$OUT/pytest_lib_ab.log"; exit 1; }
tail -1 "$OUT/pytest_lib_ab.log"
LIBS="kf2vecfsw_amd/libkf2vec_gpu_prev.so kf2vecfsw_amd/libkf2vec_gpu.so" VARIANT=${VARIANT:-1} REPEAT=${REPEAT:-3} \
  bash tools/ab_libs.sh
