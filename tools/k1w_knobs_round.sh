#!/bin/bash
# K1w knob round: parity of the wide variants, an in-process A/B of the knobs
# (nt loads, deeper ring, late return check) and bench.py lines per variant.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "variants_agree or u16_drains" > "$OUT/knobs_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/knobs_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_bench.py --variants ${AB_VARIANTS:-13,14,15,16,17} --k 7 --rounds 4 --reps 5 \
  > "$OUT/knobs_ab.json" 2> "$OUT/knobs_ab.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/knobs_ab.json'))['results']; [print('ab', k, round(v['median_ms'],4), round(v['min_ms'],4)) for k,v in d.items()]"
for v in ${BENCH_VARIANTS:-13 14 15 16 17}; do
  KF_COUNT_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --secondary-k 0 > "$OUT/knobs_bench_v$v.json" 2> "$OUT/knobs_bench_v$v.err" || exit $?
  python3 -c "import json; d=json.load(open('$OUT/knobs_bench_v$v.json')); print('bench', $v, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])"
done
