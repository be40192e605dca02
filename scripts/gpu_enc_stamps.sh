#!/bin/bash
# k_encode per-phase cycles (stamps build) and the product's cfg3 encode/decode on one chunk:
# gpurun_out/$1/{stamps,product}.log
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-encst}
mkdir -p $O
A="bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline"
MTBLX_ENC_STAMPS_PRINT=1 timeout -k 10 300 python -u $A --lib oxidized-mtbl_amd/build/libmtblx_${2:-estamps}.so > $O/stamps.log 2>&1 || exit 1
timeout -k 10 300 python -u $A > $O/product.log 2>&1 || exit 2
echo done
