#!/bin/bash
# k_snappy_lanes (MTBLX_SNAPPY_KERNEL=lanes) on the compressible 100 000-block stream: kernel
# stats and SQ counters (two PMC passes).  Outputs under gpurun_out/r03/snapprof/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03/snapprof
mkdir -p $O
export TMPDIR=/tmp MTBLX_SNAPPY_KERNEL=${MTBLX_SNAPPY_KERNEL:-lanes}
A="--blocks 100000 --tile 4 --compressible --reps 3"
P="timeout -s KILL 200 rocprofv3 --output-format csv"
$P --kernel-trace --stats -d $O/stats -o run -- python3 scripts/snappy_probe.py $A > $O/stats.log 2>&1 || exit 3
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $O/p1 -o run -- python3 scripts/snappy_probe.py $A > $O/p1.log 2>&1 || exit 4
$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d $O/p2 -o run -- python3 scripts/snappy_probe.py $A > $O/p2.log 2>&1 || exit 5
echo done
