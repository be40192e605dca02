#!/bin/bash
# adaptive walk order: full GPU parity, then A/B against the HEAD decode (cfg3, 64 KiB, cfg2)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/t_walk.log 2>&1
rc=$?; tail -2 gpurun_out/t_walk.log; [ $rc -ne 0 ] && exit $rc
LIBS="cur= base=oxidized-mtbl_amd/build/libmtblx_base.so" CFGS="cfg3 large small" bash tools/rounds/gpu_ab.sh
