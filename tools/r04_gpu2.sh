#!/bin/bash
# round 4, call 2: configs[1]/configs[3] GPU tests, prewarm variants, bench (driver args)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/r04/v2_pytest_configs.log 2>&1 &&
timeout -k 10 240 python -u tools/r04_cold.py > gpurun_out/r04/v2_cold.json 2> gpurun_out/r04/v2_cold.err &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v2_bench.json 2> gpurun_out/r04/v2_bench.err
