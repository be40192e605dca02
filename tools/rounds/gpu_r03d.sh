#!/bin/bash
# encode gather path: parity, A/B vs the LDS-assembly build, stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-run} bash tools/rounds/gpu_enc_r03.sh tests || exit $?
TAG=${TAG:-run} bash tools/rounds/gpu_enc_r03.sh ab || exit $?
O=gpurun_out/r03/enc_${TAG:-run}
timeout -k 10 300 env MTBLX_ENC_STAMPS_PRINT=1 python bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline --lib oxidized-mtbl_amd/build/libmtblx_estamps.so > $O/stamps.log 2>&1 || exit 3
grep "enc stamps" $O/stamps.log
