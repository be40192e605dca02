#!/bin/bash
# A/B on one box: GPU parity tests of the working build, then alternating bench runs of the
# HEAD build (build/libmtblx_base.so) and the working build, plus one stamps run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
val() { python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('phase_cycles_per_tile',''))" "$1" "$2"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
  tail -1 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc: stop"; exit 1; }
fi
BA="--no-cpu-baseline --no-e2e --no-crc --no-ceiling --steps 200 --warmup 20 ${BENCH_ARGS:-}"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $BA --lib oxidized-mtbl_amd/build/libmtblx_base.so > gpurun_out/ab_base$r.log 2>&1 || exit 3
  val gpurun_out/ab_base$r.log base
  timeout -k 10 300 python bench.py $BA > gpurun_out/ab_new$r.log 2>&1 || exit 3
  val gpurun_out/ab_new$r.log new
done
if [ "${STAMPS:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-crc --stamps > gpurun_out/stamps.log 2>&1 || exit 3
  val gpurun_out/stamps.log stamps
fi
if [ "${LARGE:-0}" = 1 ]; then
  for bs in 16384 65536; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --block-size $bs --blocks $((100000 * 4096 / bs)) > gpurun_out/large_$bs.log 2>&1 || exit 3
    val gpurun_out/large_$bs.log large_$bs
  done
fi
