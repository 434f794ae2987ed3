#!/bin/bash
# SQ counters of bucket_kernel<11> (two passes of <= 8 SQ counters), product library
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmc_k11_r03
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run -f csv -- python3 "$REPO/tools/ab_bench.py" --variants 19 --k ${K:-11} --rounds 1 --reps 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc" >> "$OUT/passes.txt"
  [ $rc -eq 0 ] || { echo "FATAL pass $i rc=$rc"; tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 "$REPO/tools/pmc_summary.py" "$OUT" bucket_kernel
