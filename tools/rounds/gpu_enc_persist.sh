#!/bin/bash
# Round 3: persistent k_encode workgroups (MTBLX_ENC_PERSIST=1: next ticket claimed at the block's start,
# build/libmtblx_encp.so; =2: claimed at the look-back, libmtblx_encq.so) and the block CRC with
# slicing-by-8 (MTBLX_ENC_CRC8=1, libmtblx_enc8.so) --
# encode / writer parity on the variant, then the cfg3 A/B against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03/enc_persist
mkdir -p $O
for v in encp encq enc8; do
  echo "=== t_$v ($(date +%T))"
  MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_$v.so timeout -k 10 400 python -u -m pytest tests/test_encode_gpu.py \
    -x -q --timeout 240 --timeout-method thread > $O/t_$v.log 2>&1
  rc=$?; tail -2 $O/t_$v.log; [ $rc -ne 0 ] && { echo "STOP t_$v rc=$rc"; exit $rc; }
done
LIBS="cur= encp=oxidized-mtbl_amd/build/libmtblx_encp.so encq=oxidized-mtbl_amd/build/libmtblx_encq.so enc8=oxidized-mtbl_amd/build/libmtblx_enc8.so" \
  TAG=persist bash tools/rounds/gpu_enc_r03.sh ab
