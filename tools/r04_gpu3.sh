#!/bin/bash
# round 4, call 3: full GPU suite (get_chunks rewrite, K1x for k <= 6), A/B k <= 7 vs
# the round-3 library (K1 for k <= 6), get_chunks throughput
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v3_pytest_gpu.log 2>&1 &&
for k in 3 4 5 6 7; do
  timeout -k 10 200 python -u tools/lib_ab.py --libs tools/ab/libkf2vec_head.so,tools/ab/libkf2vec_new.so --k $k \
      --rounds 4 --reps 5 > gpurun_out/r04/v3_lib_ab_k$k.json 2> gpurun_out/r04/v3_lib_ab_k$k.err || exit $?
done &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 3 > gpurun_out/r04/v3_chunks_bench.json 2> gpurun_out/r04/v3_chunks_bench.err
