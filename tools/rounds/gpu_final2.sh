#!/bin/bash
# end of round 3: the full GPU suite + smoke + the driver's bench command on the final tree, then
# the CRC grid A/B (2 vs 1 workgroups per CU)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=final2 bash tools/rounds/gpu_r03.sh tests || exit 1
TAG=final2 bash tools/rounds/gpu_r03.sh bench || exit 2
O=gpurun_out/r03/final2
for r in 1 2; do
  for v in prod crc1; do
    L=""; [ $v != prod ] && L=oxidized-mtbl_amd/build/libmtblx_$v.so
    timeout -k 10 300 env ${L:+MTBLX_LIB=$L} python scripts/crc_ab.py 0 > $O/crc_${v}_$r.log 2>&1 || exit 3
    echo "$v $(grep '^0 ' $O/crc_${v}_$r.log | head -1)"
  done
done
