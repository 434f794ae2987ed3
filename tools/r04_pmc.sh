#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass) over tools/r04_run.py.
#   LIB=<.so or empty for the product> K=11 TAG=name GROUPS_LIST=$'A B\nC D' bash tools/r04_pmc.sh
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -n "${LIB:-}" ] && export KF2VEC_GPU_LIB=$REPO/$LIB
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run -f csv -- python3 "$REPO/tools/r04_run.py" --k ${K:-11} --reps ${REPS:-2} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i [$grp] rc=$rc" >> "$OUT/passes.txt"
  case $rc in 0) ;; *) echo "FATAL pass $i rc=$rc"; tail -5 "$OUT/p$i.log"; exit $rc;; esac
done <<< "${GROUPS_LIST}"
cat "$OUT/passes.txt"
