#!/bin/bash
# per-kernel breakdown of the sparse counter at k=31 and k=16 (u64 tile 4096)
set -e
mkdir -p gpurun_out/r04/v46_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04/v46_prof -o run -f csv -- python3 $GRAFT_REPO_ROOT/tools/sparse_bench.py --genomes 64 --k 13,16,21,31 --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/r04/v46_sparse.json
