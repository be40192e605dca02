#!/bin/bash
# non-temporal DMA loads: full GPU parity, then A/B (cfg2, 64 KiB, cfg3) and the driver's bench command
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ntl.log 2>&1
rc=$?; tail -2 gpurun_out/t_ntl.log; [ $rc -ne 0 ] && exit $rc
LIBS="cur= nt0=oxidized-mtbl_amd/build/libmtblx_nt0.so ntlw3=oxidized-mtbl_amd/build/libmtblx_ntlw3.so" CFGS="small large cfg3" bash tools/rounds/gpu_ab.sh || exit 3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_ntl.log 2>&1 || exit 3
grep '^{' gpurun_out/bench_driver_ntl.log | cut -c1-200
