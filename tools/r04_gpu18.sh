#!/bin/bash
# round 4, call 18: per-kernel times of the sparse counter (k = 31 and 16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04/v18_sparse_prof" -o run -f csv -- python3 "$GRAFT_REPO_ROOT/tools/sparse_bench.py" --genomes 64 --reps 3 --k 16,31 > "$GRAFT_REPO_ROOT/gpurun_out/r04/v18_sparse_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r04/v18_sparse_prof.err")
