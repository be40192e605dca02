#!/bin/bash
# device snappy on the compressible (cfg1-style) and random (cfg2) streams: timing, kernel
# stats, SQ counters
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/snapprof
export TMPDIR=/tmp
B=${BLOCKS:-20000}
timeout -k 10 200 python3 scripts/snappy_probe.py --blocks $B --compressible > gpurun_out/snapprof/comp.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/snappy_probe.py --blocks $B > gpurun_out/snapprof/rand.log 2>&1 || exit 2
tail -1 gpurun_out/snapprof/comp.log; tail -1 gpurun_out/snapprof/rand.log
[ "${PROF:-1}" = 1 ] || exit 0
P="timeout -k 10 200 rocprofv3 --output-format csv"
$P --kernel-trace --stats -d gpurun_out/snapprof/stats -o run -- python3 scripts/snappy_probe.py --blocks $B --compressible --reps 5 > /dev/null 2>&1 || exit 3
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d gpurun_out/snapprof/p1 -o run -- python3 scripts/snappy_probe.py --blocks $B --compressible --reps 2 > /dev/null 2>&1 || exit 4
$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d gpurun_out/snapprof/p2 -o run -- python3 scripts/snappy_probe.py --blocks $B --compressible --reps 2 > /dev/null 2>&1 || exit 5
echo done
