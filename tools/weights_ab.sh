#!/bin/bash
# In-process A/B of KF_WAVE_WEIGHTS sets for one k=7 variant: tools/weights_ab.sh 20 "a,b,c,d;e,f,g,h;..."
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python tools/ab_bench.py --variants ${1:-20} --rounds ${ROUNDS:-4} --reps 5 --weights "$2" > "$OUT/ab.json" 2>&1
