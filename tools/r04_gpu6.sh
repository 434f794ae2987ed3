#!/bin/bash
# round 4, call 6: get_chunks tests + traced throughput after the arena writer and
# launch cap; weighted phase-2 rounds re-measured with byte-identical copies (noise)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "chunk" --timeout 240 --timeout-method thread \
    > gpurun_out/r04/v6_pytest_chunks.log 2>&1 &&
timeout -k 10 300 python -u tools/chunks_bench.py --genomes 32 --reps 3 > gpurun_out/r04/v6_chunks_bench.json 2> gpurun_out/r04/v6_chunks_bench.err &&
for k in 11 9; do
  timeout -k 10 240 python -u tools/lib_ab.py --libs tools/ab/libkf2vec_new.so,tools/ab/libkf2vec_rwk1x.so,tools/ab/libkf2vec_new2.so,tools/ab/libkf2vec_rwk1x2.so --k $k \
      --rounds 4 --reps 3 > gpurun_out/r04/v6_lib_ab_k${k}_rw_dup.json 2> gpurun_out/r04/v6_lib_ab_k${k}_rw_dup.err || exit $?
done
