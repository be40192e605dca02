#!/bin/bash
# A/B of the current decode library against the round-1 final kernel (build/libmtblx_r01.so),
# cfg2 (PipeSmall) and 64 KiB blocks (PipeLarge); optional GPU tests first (TESTS=1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -5 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
val() { python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'])" "$1" "$2"; }
BA="--no-cpu-baseline --no-e2e --no-crc --no-ceiling --steps 200 --warmup 20"
for r in 1 2; do
  for cfg in small large; do
    X=""; [ $cfg = large ] && X="--block-size 65536 --blocks 6250"
    timeout -k 10 300 python bench.py $BA $X --lib oxidized-mtbl_amd/build/libmtblx_r01.so > gpurun_out/abr_r01_$cfg$r.log 2>&1 || exit 3
    val gpurun_out/abr_r01_$cfg$r.log r01_$cfg
    timeout -k 10 300 python bench.py $BA $X > gpurun_out/abr_cur_$cfg$r.log 2>&1 || exit 3
    val gpurun_out/abr_cur_$cfg$r.log cur_$cfg
  done
done
