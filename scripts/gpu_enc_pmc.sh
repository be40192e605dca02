#!/bin/bash
# SQ counters of k_encode on one cfg3 chunk (two PMC passes); outputs under gpurun_out/${ROUND:-r04}/encpmc/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${ROUND:-r04}/encpmc
mkdir -p $O
export TMPDIR=/tmp
A="bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline"
P="timeout -s KILL 240 rocprofv3 --output-format csv"
$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS -d $O/p1 -o run -- python3 $A > $O/p1.log 2>&1 || exit 1
$P --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/p2 -o run -- python3 $A > $O/p2.log 2>&1 || exit 2
echo done
