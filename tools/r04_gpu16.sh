#!/bin/bash
# round 4, call 16: get_frequencies reading into reused pinned slots: CLI tests, e2e timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -k "cli" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v16_pytest_cli.log 2>&1 &&
timeout -k 10 400 python -u tools/r04_e2e_trace.py --parts 4:2,8:2,8:4,16:4 > gpurun_out/r04/v16_e2e.json 2> gpurun_out/r04/v16_e2e.err
