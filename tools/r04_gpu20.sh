#!/bin/bash
# round 4, call 20: evidence on the current tree: full GPU suite, smoke, the driver's
# bench command plain and under rocprofv3 --kernel-trace --stats, HBM traffic passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v20_pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/v20_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v20_bench.json 2> gpurun_out/r04/v20_bench.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04/v20_prof" -o run -f csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r04/v20_prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r04/v20_prof_bench.err") &&
K=7 TAG=r04/v20_traffic_k7 GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash tools/r04_pmc.sh &&
K=11 TAG=r04/v20_traffic_k11 GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash tools/r04_pmc.sh &&
python3 tools/pmc_traffic.py gpurun_out/r04/v20_traffic_k7 --kernel "k1x_kernel<7>" --k 7 --out gpurun_out/r04/v20_traffic_k7.json &&
python3 tools/pmc_traffic.py gpurun_out/r04/v20_traffic_k11 --kernel "bucket_kernel<11>" --k 11 --out gpurun_out/r04/v20_traffic_k11.json
