#!/bin/bash
# k = 9: K1x9 (two parts per span; tools/zoo/k1x9_two_part.patch applied) and its
# variants against the bucket kernel
# (KF_K9_BUCKET=1), processes alternated, configs[1]-sized batch (1,000 x 5 Mbp).
#   tools/r05_k9_ab.sh OUTFILE [ROUNDS]
# Every variant library kf2vecfsw_amd/libk9_<name>.so present (tools/build_abl.sh,
# e.g. -DKF_K9_MASKED=0) is timed too, as k1x9_<name>.
set -u
OUT=$1
ROUNDS=${2:-3}
: > "$OUT"
one() {   # one TAG [ENV=VAL ...]
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u tools/r04_run.py --k 9 --reps 5 > /tmp/k9_one.json || exit 1
  echo "{\"path\": \"$tag\", \"r\": $(cat /tmp/k9_one.json)}" >> "$OUT"
}
for i in $(seq "$ROUNDS"); do
  one k1x9 X=1
  one bucket KF_K9_BUCKET=1
  for lib in kf2vecfsw_amd/libk9_*.so; do
    [ -f "$lib" ] || continue
    v=${lib#kf2vecfsw_amd/libk9_}
    one "k1x9_${v%.so}" KF2VEC_GPU_LIB=$lib
  done
done
exit 0
