#!/bin/bash
# Static-range pair kernel (variants 10, 11): its parity tests, then one-process
# A/B against K1 (variant 1) and K1p (variant 5) with bit-for-bit output
# comparison on the 5 GB batch, then bench.py's line per variant.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "variants_agree or u16_drains" > "$OUT/pytest_k1s.log" 2>&1 || { tail -40 "$OUT/pytest_k1s.log"; exit 1; }
tail -1 "$OUT/pytest_k1s.log"
timeout -k 10 300 python3 tools/ab_bench.py --variants 1,10,11,5 --k 7 --rounds 3 --reps 5 \
  > "$OUT/k1s_ab.json" 2> "$OUT/k1s_ab.err" || { tail -5 "$OUT/k1s_ab.err"; exit 1; }
python3 -c "import json;t=open('$OUT/k1s_ab.json').read();i=t.index('{');print(t[:i].strip()[:400]);d=json.loads(t[i:]);print({k:(round(v['median_ms'],4),round(v.get('min_ms',0),4)) for k,v in d['results'].items()})"
VARIANTS="${VARIANTS:-1 10}" bash tools/bench_ab.sh
