#!/bin/bash
# One parametrised GPU-box session (replaces the per-call r0N_gpuM.sh scripts):
#   tools/gpu.sh TAG STEP [STEP...]
# Steps (each under its own time limit; the first failure ends the session):
#   tests[=EXPR]  pytest tests -m gpu [-k EXPR]        -> gpurun_out/TAG/pytest_gpu.log
#   smoke         __graft_entry__.smoke()              -> smoke.log
#   bench         the driver's bench command (--steps 20 --warmup 5)  -> bench.json
#   benchonly     bench without e2e / sparse / cpu legs -> benchonly.json
#   prof          rocprofv3 --kernel-trace --stats of `benchonly` (k=7 + k=11 only,
#                 so the per-kernel averages are the timed launches)  -> prof/
#   profsparse    rocprofv3 --kernel-trace --stats of tools/sparse_bench.py -> profsparse/
#   sparse[=K]    tools/sparse_bench.py (64 x 5 Mbp)   -> sparse.json
#   e2e           tools/e2e_bench.py                    -> e2e.json
#   cmd=...       any other command (quoted), output -> cmd_N.log
set -u
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
BENCH_ONLY="--steps 20 --warmup 5 --no-cpu --e2e-genomes 0 --sparse-k 0"
n=0
run() {   # run LIMIT OUTFILE CMD...
  local lim=$1 out=$2; shift 2
  echo "== $(date +%T) $*" >> "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$out" 2> "$out.err"
  local rc=$?
  echo "   rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "STEP FAILED rc=$rc: $*"; tail -20 "$out" "$out.err"; exit $rc; fi
}
for step in "$@"; do
  n=$((n + 1))
  case $step in
    tests) run 1100 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    tests=*) run 1100 "$OUT/pytest_gpu_$n.log" python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${step#tests=}" ;;
    smoke) run 300 "$OUT/smoke.log" python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 500 "$OUT/bench.json" python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchonly) run 300 "$OUT/benchonly.json" python -u bench.py $BENCH_ONLY ;;
    prof) (cd /tmp && export TMPDIR=/tmp && run 400 "$OUT/prof_bench.json" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -f csv -- python3 "$REPO/bench.py" $BENCH_ONLY) || exit 1 ;;
    profsparse) (cd /tmp && export TMPDIR=/tmp && run 400 "$OUT/profsparse.json" rocprofv3 --kernel-trace --stats -d "$OUT/profsparse" -o run -f csv -- python3 "$REPO/tools/sparse_bench.py" --genomes 64 --k 13,16,21,31 --reps 3) || exit 1 ;;
    sparse) run 300 "$OUT/sparse.json" python -u tools/sparse_bench.py --genomes 64 --k 13,16,17,21,31 --reps 5 ;;
    sparse=*) run 300 "$OUT/sparse_$n.json" python -u tools/sparse_bench.py --genomes 64 --k "${step#sparse=}" --reps 5 ;;
    e2e) run 300 "$OUT/e2e.json" python -u tools/e2e_bench.py ;;
    cmd=*) run 600 "$OUT/cmd_$n.log" bash -c "${step#cmd=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
