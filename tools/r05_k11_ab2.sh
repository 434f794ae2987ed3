#!/bin/bash
# Round 5, k=11 with two rank replicas (the new default): k >= 9 parity tests on
# the product library, an in-process A/B against R = 1 and the phase-2 knobs
# (equal round weights, both groups pre-issued, wave priorities), and the
# phase-1-only LDS counters of the R = 2 build.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05/k11ab2}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
L=kf2vecfsw_amd
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "bucket or configs4 or k12 or large_k or count_matrix" > "$OUT/pytest_bucket.log" 2>&1 || { tail -20 "$OUT/pytest_bucket.log"; exit 1; }
tail -1 "$OUT/pytest_bucket.log"
timeout -k 10 300 python3 -u tools/lib_ab.py --libs $L/libkf2vec_gpu.so,$L/libkf2vec_gpu_rl0.so,$L/libkf2vec_gpu_rw0.so,$L/libkf2vec_gpu_pre2.so,$L/libkf2vec_gpu_prio3.so \
  --k 11 --rounds 4 --reps 5 > "$OUT/ab_k11.json" 2> "$OUT/ab_k11.err" || { tail -5 "$OUT/ab_k11.err"; exit 1; }
LIB=$L/libkf2vec_gpu_abl8rl1.so K=11 TAG=$TAG/pmc_abl8rl1 \
  GROUPS_LIST="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
  bash tools/r04_pmc.sh || exit 1
echo done
