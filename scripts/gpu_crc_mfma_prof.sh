#!/bin/bash
# k_crc32c_mfma on the cfg2 batch: tests, A/B timing vs the VALU kernel, kernel trace, SQ counters
# (separate --pmc passes, each under its own time limit), FETCH_SIZE.  Output: gpurun_out/$1/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-crcm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_crc_mfma_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/crc_ab.py ${AB:-mfma lanes} > $O/crc_ab.log 2>&1 || exit 2
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
P="rocprofv3 --output-format csv"
timeout -k 10 120 $P --kernel-trace --stats -d $O/stats -o run -- python3 scripts/crc_probe.py > $O/stats.log 2>&1 || exit 3
timeout -s KILL 90 $P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -o run -- python3 scripts/crc_probe.py 100000 3 > $O/p1.log 2>&1 || exit 4
timeout -s KILL 90 $P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d $O/p2 -o run -- python3 scripts/crc_probe.py 100000 3 > $O/p2.log 2>&1 || exit 5
timeout -s KILL 90 $P --pmc FETCH_SIZE -d $O/p3 -o run -- python3 scripts/crc_probe.py 100000 3 > $O/p3.log 2>&1 || exit 6
echo done
