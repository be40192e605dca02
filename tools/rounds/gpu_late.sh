#!/bin/bash
# PipeLarge late-walk schedule: parity on the 64 KiB cases, then A/B (cfg3, 64 KiB / 16 B keys)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_cfg4_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "key_tails or 64k or cfg4 or large or workspace" > gpurun_out/t_late.log 2>&1
rc=$?; tail -4 gpurun_out/t_late.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks 100000 --stamps --no-cpu-baseline > gpurun_out/stamps_cfg3_late.log 2>&1 || exit 3
LIBS="${LIBS:-cur= late0=oxidized-mtbl_amd/build/libmtblx_late0.so lc=oxidized-mtbl_amd/build/libmtblx_lc.so}" CFGS="${CFGS:-cfg3 large}" bash tools/rounds/gpu_ab.sh
