#!/bin/bash
# round 4, call 25: FASTA record index on the device (kf_index_fasta): its tests, the CLI
# tests, e2e timeline and the bench's e2e object
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -k "index or cli or toy" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v25_pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/r04_e2e_trace.py --parts 8:2,8:4 > gpurun_out/r04/v25_e2e.json 2> gpurun_out/r04/v25_e2e.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --secondary-k 0 --sparse-k 0 > gpurun_out/r04/v25_bench_e2e.json 2> gpurun_out/r04/v25_bench_e2e.err &&
timeout -k 10 300 python -u tools/lib_ab.py --libs tools/ablib/libkf2vec_p1.so,tools/ablib/libkf2vec_abl1.so,tools/ablib/libkf2vec_abl9.so,tools/ablib/libkf2vec_p2.so --k 11 \
    --rounds 4 --reps 3 > gpurun_out/r04/v25_lib_ab_k11_flush.json 2> gpurun_out/r04/v25_lib_ab_k11_flush.err
