#!/bin/bash
# k_snappy_lanes far copies: cached loads after whole-line visibility (product) vs device-coherent
# dword loads (faratom); parity under lanes routing, timing, per-path counters
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03/far
mkdir -p $O
export TMPDIR=/tmp MTBLX_SNAPPY_KERNEL=lanes
A="--compressible --blocks 100000 --tile 4"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_snappy_gpu.py tests/test_pipe_gpu.py > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
echo "tests: $(tail -1 $O/t.log)"
for r in 1 2; do
  for v in prod faratom; do
    L=""; [ $v != prod ] && L=oxidized-mtbl_amd/build/libmtblx_$v.so
    timeout -k 10 300 env ${L:+MTBLX_LIB=$L} python scripts/snappy_probe.py $A > $O/${v}_$r.log 2>&1 || exit 2
    echo "$v $(grep decompress $O/${v}_$r.log)"
  done
done
timeout -k 10 300 env MTBLX_LIB=oxidized-mtbl_amd/mtblx/libmtblx_snapstamps.so python scripts/snappy_probe.py $A > $O/stamps.log 2>&1 || exit 3
grep "lanes:\|decompress" $O/stamps.log
