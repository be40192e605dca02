#!/bin/bash
# memory-pipeline counters of the CRC kernels (0 and 5): gpurun_out/r03/crcprof/k*/p3
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03/crcprof
mkdir -p $O
P="rocprofv3 --output-format csv"
S3="TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES GRBM_GUI_ACTIVE"
for k in ${KS:-0 5}; do
  export MTBLX_CRC_KERNEL=$k
  timeout -s KILL 90 $P --pmc $S3 -d $O/k$k/p3 -o run -- python3 scripts/crc_probe.py 100000 3 > $O/k${k}_p3.log 2>&1 || exit 2
done
echo ALL DONE
