#!/bin/bash
# k_encode: parity tests, then per-phase stamps of two builds and the product cfg3 line.
# usage: gpu_enc_ab.sh OUT STAMPS_A STAMPS_B  (build names under oxidized-mtbl_amd/build/libmtblx_<name>.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-encab}
mkdir -p $O
A="bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_encode_gpu.py tests/test_writer_gpu.py > $O/tests.log 2>&1 || exit 1
for v in ${2:-estamps} ${3:-estamps0}; do
  MTBLX_ENC_STAMPS_PRINT=1 timeout -k 10 300 python -u $A --lib oxidized-mtbl_amd/build/libmtblx_$v.so > $O/stamps_$v.log 2>&1 || exit 2
done
timeout -k 10 300 python -u $A > $O/product.log 2>&1 || exit 3
echo done
