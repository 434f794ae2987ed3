#!/bin/bash
# k=7 pair-kernel session: focused parity tests, then A/B timing of the k=7 variants
# (1 = forward-histogram kernel; 5/6/7 = pair kernel, ring 6/4/8), schedule
# settings (KF_PAIR_SCHED) and a cycle profile.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-pair or k7_kernel or toy or random_fasta_all_k or one_large or many_small or device_synth or deterministic or end_at_every or arbitrary}" \
  > "$OUT/pytest_pair.log" 2>&1 || { tail -30 "$OUT/pytest_pair.log"; exit 1; }
tail -2 "$OUT/pytest_pair.log"
fi
timeout -k 10 300 python -u tools/ab_bench.py --variants ${VARIANTS:-1,5,6,7} --k 7 --rounds 3 --reps 5 > "$OUT/ab_pair.json" 2>> "$OUT/ab.err" || { cat "$OUT/ab_pair.json"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/ab_pair.json'));print({k:round(v['median_ms'],4) for k,v in d['results'].items()})"
for S in ${SCHEDS:-}; do
  KF_PAIR_SCHED=$S timeout -k 10 200 python -u tools/ab_bench.py --variants 5 --k 7 --rounds 2 --reps 5 > "$OUT/ab_sched.json" 2>> "$OUT/ab.err" || { cat "$OUT/ab_sched.json"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ab_sched.json'));print('$S', {k:round(v['median_ms'],4) for k,v in d['results'].items()})"
done
KF_COUNT_PROFILE=1 KF_COUNT_VARIANT=${PROF_VARIANT:-5} timeout -k 10 120 python -u tools/ab_bench.py --variants ${PROF_VARIANT:-5} --k 7 --rounds 1 --reps 1 > "$OUT/prof_pair.log" 2>&1
head -18 "$OUT/prof_pair.log"
