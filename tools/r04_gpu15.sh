#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 200 python -u tools/sparse_debug.py > gpurun_out/r04/v15_sparse_debug.txt 2>&1
