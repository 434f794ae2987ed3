#!/bin/bash
# pair kernel: parity (pair variants), A/B vs variant 1, stream-only ablation, cycle profile
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pair or k7_kernel" > "$OUT/pytest_pair.log" 2>&1 || { tail -30 "$OUT/pytest_pair.log"; exit 1; }
tail -1 "$OUT/pytest_pair.log"
timeout -k 10 300 python -u tools/ab_bench.py --variants 1,5,6,7 --k 7 --rounds 3 --reps 5 > "$OUT/ab_pair.json" 2>> "$OUT/ab.err" || exit 1
python3 -c "import json;d=json.load(open('$OUT/ab_pair.json'));print({k:round(v['median_ms'],4) for k,v in d['results'].items()})"
for S in ${SCHEDS:-}; do
  KF_PAIR_SCHED=$S timeout -k 10 200 python -u tools/ab_bench.py --variants 5 --k 7 --rounds 2 --reps 5 > "$OUT/ab_sched.json" 2>> "$OUT/ab.err" || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab_sched.json'));print('$S', {k:round(v['median_ms'],4) for k,v in d['results'].items()})"
done
KF2VEC_GPU_LIB=$GRAFT_REPO_ROOT/kf2vecfsw_amd/libkf2vec_gpu_pabl3.so timeout -k 10 200 python -u tools/ab_bench.py --variants 5 --k 7 --rounds 2 --reps 5 > "$OUT/ab_abl3.json" 2>> "$OUT/ab.err" || exit 1
python3 -c "import json;d=json.load(open('$OUT/ab_abl3.json'));print('stream-only', {k:round(v['median_ms'],4) for k,v in d['results'].items()})"
KF_COUNT_PROFILE=1 timeout -k 10 120 python -u tools/ab_bench.py --variants 5 --k 7 --rounds 1 --reps 1 > "$OUT/prof_pair.log" 2>&1
grep -v amdgpu.ids "$OUT/prof_pair.log" | head -18
