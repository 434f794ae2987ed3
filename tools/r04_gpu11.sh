#!/bin/bash
# round 4, call 11: get_chunks with u16 count rows on a copy stream of their own;
# chunk tests, traced throughput; smoke with the sparse counter
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -k "chunk" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v11_pytest_chunks.log 2>&1 &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 5 > gpurun_out/r04/v11_chunks_bench.json 2> gpurun_out/r04/v11_chunks_bench.err &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/v11_smoke.log 2>&1
