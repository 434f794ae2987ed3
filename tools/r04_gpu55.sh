#!/bin/bash
# round 4, call 55: evidence on the final tree: full GPU suite, smoke, the driver's
# bench command plain and under rocprofv3 --kernel-trace --stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v55_pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/v55_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v55_bench.json 2> gpurun_out/r04/v55_bench.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04/v55_prof" -o run -f csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r04/v55_prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r04/v55_prof_bench.err")
