#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes for the bench workload at each k of K_LIST
# (default 7 11) -> gpurun_out/traffic_k<k>.json and profiles/<round>/ (bench.py reads them).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
ROUND=${ROUND:-r02}
V7=${V7:-19}   # the k=7 default variant (KF_COUNT_VARIANT)
V8=${V8:-24}   # the k=8 default variant
for k in ${K_LIST:-7 11}; do
  V=$V7; [ $k -eq 8 ] && V=$V8
  if [ $k -le 8 ]; then KN="count_kernel<$k, $V>"; else KN="bucket_kernel<$k>"; fi
  PMC_TAG=pmc_k$k VARIANT=$V GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' AB_ARGS="--k $k" bash "$REPO/tools/pmc_variant.sh" || exit $?
  python3 "$REPO/tools/pmc_traffic.py" "$REPO/gpurun_out/pmc_k$k" --kernel "$KN" --k $k \
      --out "$REPO/gpurun_out/traffic_k$k.json" || exit $?
  mkdir -p "$REPO/profiles/$ROUND" && cp "$REPO/gpurun_out/traffic_k$k.json" "$REPO/profiles/$ROUND/"
done
