#!/bin/bash
# k_snappy_lanes: a far copy's (snpf1) / also a long literal's (snpf2) next chunk loaded one
# iteration ahead (MTBLX_LANE_FAR_PF) against the product: parity on each variant, then timing
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03/snap_pf
mkdir -p $O
export TMPDIR=/tmp
A="--compressible --blocks 100000 --tile 4"
for v in snpf1 snpf2; do
  MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_snappy_gpu.py > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $O/t_$v.log)"
done
for r in 1 2; do
  for v in prod snpf1 snpf2; do
    L=""; [ $v != prod ] && L=oxidized-mtbl_amd/build/libmtblx_$v.so
    timeout -k 10 300 env ${L:+MTBLX_LIB=$L} python scripts/snappy_probe.py $A > $O/${v}_$r.log 2>&1 || exit 2
    echo "$v $(grep decompress $O/${v}_$r.log)"
  done
done
