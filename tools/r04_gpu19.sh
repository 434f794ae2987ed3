#!/bin/bash
# round 4, call 19: sparse counter with LDS-atomic histograms and a 32-byte-per-thread emit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r04/v19_pytest_sparse.log 2>&1 &&
timeout -k 10 200 python -u tools/sparse_bench.py --genomes 64 --reps 5 \
    > gpurun_out/r04/v19_sparse_bench.json 2> gpurun_out/r04/v19_sparse_bench.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04/v19_sparse_prof" -o run -f csv -- python3 "$GRAFT_REPO_ROOT/tools/sparse_bench.py" --genomes 64 --reps 3 --k 16,31 > "$GRAFT_REPO_ROOT/gpurun_out/r04/v19_sparse_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r04/v19_sparse_prof.err")
