#!/bin/bash
# Round evidence: GPU tests, smoke, the default bench line, the driver's 20-step line, cfg3 and
# cfg4 lines, a kernel-trace stats run.  Outputs under gpurun_out/final/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_default 600 python bench.py
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e
fi
if [ "$MODE" = all ] || [ "$MODE" = configs ]; then
  step cfg3 900 python bench.py --config cfg3 --no-cpu-baseline
  step cfg4 900 python bench.py --config cfg4 --no-cpu-baseline
fi
echo ALL DONE
