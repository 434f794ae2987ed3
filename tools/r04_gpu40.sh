#!/bin/bash
# round 4, call 40: evidence on the final tree: full GPU suite, smoke, the driver's
# bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v40_pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/v40_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v40_bench.json 2> gpurun_out/r04/v40_bench.err
