#!/bin/bash
# round 4, call 24: bench line with the sparse object (short run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --secondary-k 0 --e2e-genomes 0 > gpurun_out/r04/v24_bench_sparse.json 2> gpurun_out/r04/v24_bench_sparse.err
