#!/bin/bash
# k_snappy_lanes ring size A/B: 256 B x 256 lanes (product), 512 B x 128 lanes, 1 KiB x 64 lanes
# per workgroup; parity under each, timing, and the per-path counters (stamps builds)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03/ring
mkdir -p $O
export TMPDIR=/tmp MTBLX_SNAPPY_KERNEL=lanes
A="--compressible --blocks 100000 --tile 4"
for v in r128 r256; do
  timeout -k 10 300 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_$v.so python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_snappy_gpu.py > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/t_$v.log)"
done
for r in 1 2; do
  for v in prod r128 r256; do
    L=""; [ $v != prod ] && L=oxidized-mtbl_amd/build/libmtblx_$v.so
    timeout -k 10 300 env ${L:+MTBLX_LIB=$L} python scripts/snappy_probe.py $A > $O/${v}_$r.log 2>&1 || exit 2
    echo "$v $(grep decompress $O/${v}_$r.log)"
  done
done
for v in r128s r256s; do
  timeout -k 10 300 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_$v.so python scripts/snappy_probe.py $A > $O/$v.log 2>&1 || exit 3
  echo "$v $(grep lanes: $O/$v.log)"
done
