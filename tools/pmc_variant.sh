#!/bin/bash
# PMC passes on tools/ab_bench.py for one KF_COUNT_VARIANT (VARIANT env), counters from GROUPS_LIST.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${PMC_TAG:-pmcv$VARIANT}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run -f csv -- python3 "$REPO/tools/ab_bench.py" --variants $VARIANT --rounds 1 --reps 2 ${AB_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i [$grp] rc=$rc" >> "$OUT/passes.txt"
  case $rc in 0) ;; *) echo "FATAL pass $i rc=$rc"; exit $rc;; esac
done <<< "${GROUPS_LIST}"
cat "$OUT/passes.txt"
