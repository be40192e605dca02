#!/bin/bash
# writer idle-sleep A/B of k_snappy_lanes (product = 8; variants ws2, ws20), compressible stream
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03/ws
mkdir -p $O
export TMPDIR=/tmp MTBLX_SNAPPY_KERNEL=lanes
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_snappy_gpu.py > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for v in prod ws2 ws20; do
    L=""; [ $v != prod ] && L=oxidized-mtbl_amd/build/libmtblx_$v.so
    timeout -k 10 300 env ${L:+MTBLX_LIB=$L} python scripts/snappy_probe.py --compressible --blocks 100000 --tile 4 > $O/${v}_$r.log 2>&1 || exit 2
    echo "$v $(grep decompress $O/${v}_$r.log)"
  done
done
