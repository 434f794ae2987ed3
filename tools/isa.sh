#!/bin/bash
# ISA + resource usage of one k=7 count_kernel variant: tools/isa.sh 22 [extra hipcc flags]
V=${1:-22}; shift
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -DKF_QUICK_ISA=$V "$@" \
  -Rpass-analysis=kernel-resource-usage /root/repo/kf2vecfsw_amd/csrc/kf_count.hip -o /tmp/isa_v$V.s 2> /tmp/isa_v$V.res
grep -E "VGPRs|SGPRs|Scratch|Occupancy" /tmp/isa_v$V.res | grep -v "^$" | sed 's/.*remark: *//' | sort -u
