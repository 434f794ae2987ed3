#!/bin/bash
# Build the working tree's HIP library with extra hipcc flags into OUT
# (profiling ablations, e.g. -DKF_BK_ABL=1; not for correctness runs).
#   tools/build_abl.sh kf2vecfsw_amd/libkf2vec_gpu_abl1.so -DKF_BK_ABL=1
set -eu
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp -r "$ROOT/kf2vecfsw_amd" "$ROOT/include" "$TMP/"
rm -rf "$TMP/kf2vecfsw_amd/_build" "$TMP"/kf2vecfsw_amd/*.so
KF_HIPCC_FLAGS="$*" python3 "$TMP/kf2vecfsw_amd/build.py" --force > /dev/null
cp "$TMP/kf2vecfsw_amd/libkf2vec_gpu.so" "$ROOT/$OUT"
rm -rf "$TMP"
echo "$OUT"
