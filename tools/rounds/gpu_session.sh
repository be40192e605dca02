#!/bin/bash
# One gpurun session: GPU parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first crash/timeout (exit >= 124 or signal); a plain test failure (exit 1)
# still lets the bench run so we see numbers.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
