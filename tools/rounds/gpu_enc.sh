#!/bin/bash
# encode changes: GPU parity (encode / writer / cfg3-shaped), phase stamps, cfg3 encode rate x2
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_encode_gpu.py tests/test_writer_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_enc.log 2>&1
rc=$?; tail -3 gpurun_out/t_enc.log; [ $rc -ne 0 ] && exit $rc
MTBLX_ENC_STAMPS_PRINT=1 timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline --lib oxidized-mtbl_amd/build/libmtblx_estamps.so > gpurun_out/estamps.log 2>&1 || exit 3
grep "enc stamps" gpurun_out/estamps.log
LIBS="${LIBS:-cur=}" bash tools/rounds/gpu_ab_enc.sh
