#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/crcprof
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/crcprof/counters.txt 2>&1 || true
P="timeout -k 10 120 rocprofv3 --output-format csv"
$P --kernel-trace --stats -d gpurun_out/crcprof/stats -o run -- python3 scripts/crc_probe.py > gpurun_out/crcprof/stats.log 2>&1 || exit 1
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/crcprof/p1 -o run -- python3 scripts/crc_probe.py 100000 3 > gpurun_out/crcprof/p1.log 2>&1 || exit 2
$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM -d gpurun_out/crcprof/p2 -o run -- python3 scripts/crc_probe.py 100000 3 > gpurun_out/crcprof/p2.log 2>&1 || exit 3
$P --pmc FETCH_SIZE -d gpurun_out/crcprof/p3 -o run -- python3 scripts/crc_probe.py 100000 3 > gpurun_out/crcprof/p3.log 2>&1 || exit 4
find gpurun_out/crcprof -name "*.csv" | sort
