#!/bin/bash
# round 4, call 13: e2e read-ahead depth sweep (parts:ahead)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u tools/r04_e2e_trace.py --parts 8:2,8:4,8:8,16:4,16:8,16:16,32:16 > gpurun_out/r04/v13_e2e_ahead.json 2> gpurun_out/r04/v13_e2e_ahead.err
