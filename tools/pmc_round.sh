#!/bin/bash
# PMC counter passes (kernel-trace only, one counter group per pass) over the bench workload.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ "${LIST:-0}" = 1 ]; then timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; fi
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu --verify 0"}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run -f csv -- python3 "$REPO/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i [$grp] rc=$rc" >> "$OUT/passes.txt"
  case $rc in 0) ;; *) echo "FATAL pass $i rc=$rc"; exit $rc;; esac
done <<< "${GROUPS_LIST}"
cat "$OUT/passes.txt"
