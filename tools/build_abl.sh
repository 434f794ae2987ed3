#!/bin/bash
# Build a profiling variant of the HIP library into OUT: the ablation sources
# (kf2vecfsw_amd/build.py --ablation: tools/zoo/*_ablations.patch applied) with
# extra hipcc flags (e.g. -DKF_BK_ABL=1, -DKF_K9_ABL=2); never for correctness runs.
#   tools/build_abl.sh kf2vecfsw_amd/libkf2vec_gpu_k9abl1.so -DKF_K9_ABL=1
set -eu
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
KF_HIPCC_FLAGS="$*" python3 -c "
import sys; sys.path.insert(0, '.')
from kf2vecfsw_amd import build as B
print(B.build(ablation=True, out='$ROOT/$OUT'))"
