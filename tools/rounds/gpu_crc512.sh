#!/bin/bash
# CRC grid shape: 512-thread workgroups, two per CU (crc512) against the product (1024 threads,
# one per CU); parity of the variant, then two alternations of scripts/crc_ab.py
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03/crc512
mkdir -p $O
export TMPDIR=/tmp
L=oxidized-mtbl_amd/build/libmtblx_crc512.so
MTBLX_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_decode_gpu.py::test_crc32c_blocks_vs_oracle" "tests/test_decode_gpu.py::test_fused_verify_decode" > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
echo "tests: $(tail -n 1 $O/t.log)"
for r in 1 2; do
  for v in prod crc512; do
    timeout -k 10 300 env $([ $v != prod ] && echo MTBLX_LIB=$L) python scripts/crc_ab.py 0 > $O/${v}_$r.log 2>&1 || exit 2
    echo "$v $(grep '^0 ' $O/${v}_$r.log | head -1)"
  done
done
