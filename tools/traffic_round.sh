#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes for the bench workload at each k of K_LIST
# (default 7 11) -> gpurun_out/traffic_k<k>.json and profiles/<round>/ (bench.py reads them).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
ROUND=${ROUND:-r03}
for k in ${K_LIST:-7 11}; do
  if [ $k -le 6 ]; then KN="k1_kernel<$k>"; elif [ $k -le 8 ]; then KN="k1x_kernel<$k>"; else KN="bucket_kernel<$k>"; fi
  PMC_TAG=pmc_k$k VARIANT=19 GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' AB_ARGS="--k $k" bash "$REPO/tools/pmc_variant.sh" || exit $?
  python3 "$REPO/tools/pmc_traffic.py" "$REPO/gpurun_out/pmc_k$k" --kernel "$KN" --k $k \
      --out "$REPO/gpurun_out/traffic_k$k.json" || exit $?
  mkdir -p "$REPO/profiles/$ROUND" && cp "$REPO/gpurun_out/traffic_k$k.json" "$REPO/profiles/$ROUND/"
done
