#!/bin/bash
# round 4, call 26: get_frequencies with each batch's H2D issued by its reader on a copy
# stream: CLI tests, e2e timeline, bench e2e
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_parity.py -m gpu -x -v -k "index or cli" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v26_pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/r04_e2e_trace.py --parts 8:2,8:4,16:4 > gpurun_out/r04/v26_e2e.json 2> gpurun_out/r04/v26_e2e.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --secondary-k 0 --sparse-k 0 > gpurun_out/r04/v26_bench_e2e.json 2> gpurun_out/r04/v26_bench_e2e.err
