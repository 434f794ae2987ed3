#!/bin/bash
# Build the HIP library of git revision REV into OUT (for process-level A/B runs
# against the working tree: KF2VEC_ALLOW_FOREIGN_LIB=1 KF2VEC_GPU_LIB=OUT python tools/...;
# _native refuses a library built from other sources unless that is set).
#   tools/build_rev.sh HEAD~1 kf2vecfsw_amd/libkf2vec_gpu_prev.so
set -eu
REV=$1; OUT=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" kf2vecfsw_amd include | tar -x -C "$TMP"
python3 "$TMP/kf2vecfsw_amd/build.py" --force > /dev/null
cp "$TMP/kf2vecfsw_amd/libkf2vec_gpu.so" "$OUT"
rm -rf "$TMP"
echo "$OUT"
