#!/bin/bash
# end of round 3, final tree (CRC grid one workgroup per CU, losing variants removed): the full
# GPU suite incl. the spilling build, smoke, the driver's bench command, the product CRC timing
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=final3 bash tools/rounds/gpu_r03.sh tests || exit 1
TAG=final3 bash tools/rounds/gpu_r03.sh bench || exit 2
O=gpurun_out/r03/final3
timeout -k 10 300 python scripts/crc_ab.py 0 > $O/crc_prod.log 2>&1 || exit 3
echo "prod $(grep '^0 ' $O/crc_prod.log | head -1)"
TAG=final3 bash tools/rounds/gpu_r03.sh spill || exit 4
