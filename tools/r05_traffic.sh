#!/bin/bash
# HBM traffic per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per
# pass) of the product kernels at k=7 and k=11 on the bench batch.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
for k in 7 11; do
  K=$k TAG=r05/traffic_k$k GROUPS_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash "$REPO/tools/r04_pmc.sh" || exit 1
done
echo done
