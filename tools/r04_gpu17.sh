#!/bin/bash
# round 4, call 17: get_frequencies with pinned slots + ramped first batches: e2e timeline, bench e2e
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "cli" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v17_pytest_cli.log 2>&1 &&
timeout -k 10 400 python -u tools/r04_e2e_trace.py --parts 4:2,8:2,8:4,16:4 > gpurun_out/r04/v17_e2e.json 2> gpurun_out/r04/v17_e2e.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --secondary-k 0 > gpurun_out/r04/v17_bench_e2e.json 2> gpurun_out/r04/v17_bench_e2e.err
