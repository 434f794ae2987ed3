#!/bin/bash
# round 4, call 12: get_frequencies with per-file H2D on a copy stream (overlaps the
# batch's reading): CLI tests, e2e timeline at 4/8/16 parts, bench e2e object
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "cli" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v12_pytest_cli.log 2>&1 &&
timeout -k 10 300 python -u tools/r04_e2e_trace.py --parts 4,8,16 > gpurun_out/r04/v12_e2e_trace.json 2> gpurun_out/r04/v12_e2e_trace.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --secondary-k 0 > gpurun_out/r04/v12_bench_e2e.json 2> gpurun_out/r04/v12_bench_e2e.err
