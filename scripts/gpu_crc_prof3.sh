#!/bin/bash
# k_crc32c_blocks (MTBLX_CRC_KERNEL=0) vs k_crc32c_lp (3) on the cfg2 batch: kernel trace + two
# SQ counter passes each, and the counter list of the box.  gpurun_out/r03/crcprof/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03/crcprof
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
P="rocprofv3 --output-format csv"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
S2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM"
for k in 0 3; do
  export MTBLX_CRC_KERNEL=$k
  timeout -k 10 120 $P --kernel-trace --stats -d $O/k$k/stats -o run -- python3 scripts/crc_probe.py 100000 20 > $O/k${k}_stats.log 2>&1 || exit 1
  timeout -s KILL 90 $P --pmc $S1 -d $O/k$k/p1 -o run -- python3 scripts/crc_probe.py 100000 3 > $O/k${k}_p1.log 2>&1 || exit 2
  timeout -s KILL 90 $P --pmc $S2 -d $O/k$k/p2 -o run -- python3 scripts/crc_probe.py 100000 3 > $O/k${k}_p2.log 2>&1 || exit 3
done
echo ALL DONE
