#!/bin/bash
# round 4, call 5: weighted phase-2 rounds A/B (k = 9..12), the driver's bench command
# plain and under rocprofv3 --kernel-trace --stats, HBM traffic passes at k = 7 and 11
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
for k in 11 9 10 12; do
  timeout -k 10 240 python -u tools/lib_ab.py --libs tools/ab/libkf2vec_new.so,tools/ab/libkf2vec_rwk1x.so,tools/ab/libkf2vec_rw6543.so,tools/ab/libkf2vec_rw3322.so --k $k \
      --rounds 4 --reps 3 > gpurun_out/r04/v5_lib_ab_k${k}_rw.json 2> gpurun_out/r04/v5_lib_ab_k${k}_rw.err || exit $?
done &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04/v5_bench.json 2> gpurun_out/r04/v5_bench.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04/v5_prof" -o run -f csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r04/v5_prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r04/v5_prof_bench.err") &&
K=7 TAG=r04/v5_traffic_k7 GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash tools/r04_pmc.sh &&
K=11 TAG=r04/v5_traffic_k11 GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash tools/r04_pmc.sh &&
python3 tools/pmc_traffic.py gpurun_out/r04/v5_traffic_k7 --kernel "k1x_kernel<7>" --k 7 --out gpurun_out/r04/traffic_k7.json &&
python3 tools/pmc_traffic.py gpurun_out/r04/v5_traffic_k11 --kernel "bucket_kernel<11>" --k 11 --out gpurun_out/r04/traffic_k11.json
