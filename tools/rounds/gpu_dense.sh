#!/bin/bash
# dense key-tail copy: parity tests, A/B vs the HEAD decode (cfg3, 64 KiB, cfg2), cfg3 stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "key_tails or 64k or builder or mutated" > gpurun_out/t_dense.log 2>&1
rc=$?; tail -5 gpurun_out/t_dense.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks 100000 --stamps --no-cpu-baseline > gpurun_out/stamps_cfg3.log 2>&1 || exit 3
LIBS="cur= base=oxidized-mtbl_amd/build/libmtblx_base.so" CFGS="${CFGS:-cfg3 large small}" bash tools/rounds/gpu_ab.sh
