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
#   alt=K:REPS:ROUNDS:V1,V2  processes alternated (one per library and repetition,
#                 tools/r04_run.py at k=K): kf2vecfsw_amd/libkf2vec_gpu_<V>.so, "product"
#                 = the product library; ENV:NAME=VAL entries instead run the product
#                 with that variable (e.g. ENV:KF_K9_BUCKET=1 with the ablation build)
#                 -> alt_N.jsonl (the round-5 k11 / k9 / coop / db / barrier A/Bs)
#   libab=K:V1,V2 in-process A/B of library variants (tools/lib_ab.py) -> libab_N.json
#   pmc=K:LIB:G1;G2  rocprofv3 --pmc passes, one counter group per pass (';' between
#                 groups, ' ' inside one), over tools/r04_run.py at k=K with LIB
#                 ("product" or a library file name) -> pmc_N/
#   traffic=K     FETCH_SIZE / WRITE_SIZE passes at k=K -> traffic_kK/ (tools/pmc_traffic.py)
#   sparsealt=V1,V2  tools/sparse_bench.py per library variant, alternated twice -> sparsealt_N.jsonl
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
    alt=*)
      IFS=: read -r ak areps arounds alibs <<< "${step#alt=}"
      for rep in $(seq "$arounds"); do
        for v in ${alibs//,/ }; do
          envs=(); lib=""
          case $v in
            product) ;;
            ENV:*) envs=("${v#ENV:}"); lib=kf2vecfsw_amd/libkf2vec_gpu_ablation.so ;;
            *) lib=kf2vecfsw_amd/libkf2vec_gpu_$v.so ;;
          esac
          run 150 "$OUT/alt_p.json" env ${lib:+KF2VEC_ALLOW_FOREIGN_LIB=1 KF2VEC_GPU_LIB=$REPO/$lib} "${envs[@]}" \
            python3 -u tools/r04_run.py --k "$ak" --reps "$areps"
          python3 -c "import json,statistics,sys;x=json.loads(open('$OUT/alt_p.json').read().strip().splitlines()[-1]);print(json.dumps({'variant':sys.argv[1],'k':$ak,'median_ms':statistics.median(x['ms'][2:]),'ms':x['ms'],'ok':x.get('totals_analytic')}))" "$v" >> "$OUT/alt_$n.jsonl"
        done
      done ;;
    libab=*)
      IFS=: read -r lk llibs <<< "${step#libab=}"
      libs=""
      for v in ${llibs//,/ }; do
        if [ "$v" = product ]; then libs="$libs,kf2vecfsw_amd/libkf2vec_gpu.so"; else libs="$libs,kf2vecfsw_amd/libkf2vec_gpu_$v.so"; fi
      done
      libs=${libs#,}
      run 300 "$OUT/libab_$n.json" python3 -u tools/lib_ab.py --libs "$libs" --k "$lk" --rounds 4 --reps 5 ;;
    pmc=*)
      IFS=: read -r pk plib pgroups <<< "${step#pmc=}"
      [ "$plib" = product ] && plib=""
      (LIB=${plib:+kf2vecfsw_amd/$plib} K=$pk TAG=${TAG}/pmc_$n GROUPS_LIST="${pgroups//;/$'\n'}" \
        timeout -k 10 900 bash tools/r04_pmc.sh > "$OUT/pmc_$n.log" 2>&1) || { tail -5 "$OUT/pmc_$n.log"; exit 1; } ;;
    traffic=*)
      tk=${step#traffic=}
      (K=$tk TAG=${TAG}/traffic_k$tk GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' timeout -k 10 600 bash tools/r04_pmc.sh \
        > "$OUT/traffic_k$tk.log" 2>&1) || { tail -5 "$OUT/traffic_k$tk.log"; exit 1; } ;;
    sparsealt=*)
      for rep in 1 2; do
        for v in product ${step#sparsealt=}; do
          lib=""; [ "$v" = product ] || lib=kf2vecfsw_amd/libkf2vec_gpu_$v.so
          run 200 "$OUT/sp_p.json" env ${lib:+KF2VEC_GPU_LIB=$REPO/$lib} python3 -u tools/sparse_bench.py --genomes 64 --k 13,16,31 --reps 5
          python3 -c "import json,sys;d=json.loads(open('$OUT/sp_p.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':sys.argv[1],'ms':{k:v['ms'] for k,v in d['k'].items()},'ok':[v['totals_ok'] for v in d['k'].values()]}))" "$v" >> "$OUT/sparsealt_$n.jsonl"
        done
      done ;;
    cmd=*) run 600 "$OUT/cmd_$n.log" bash -c "${step#cmd=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
