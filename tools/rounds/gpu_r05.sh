#!/bin/bash
# Round 5 GPU session: MODE = tests | smoke | bench | cfg3 | bounds | all (tests+smoke+bench).
# Outputs under gpurun_out/r05/<TAG>/.  Every GPU step has its own time limit; a step that
# times out, aborts or faults ends the call (test failures, rc 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05/${TAG:-run}
mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "$O/$name.log" | cut -c1-600
  if [ $rc -eq 1 ] && [ "${name%%_*}" = gpu ]; then echo "(test failures: going on)"; return 0; fi
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for MODE in ${MODES:-all}; do
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-}
fi
if [ "$MODE" = all ] || [ "$MODE" = smoke ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
fi
if [ "$MODE" = bounds ]; then   # the bounds-checked diagnostic library under the whole GPU suite
  step gpu_bounds 1150 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_bounds.so MTBLX_BOUNDS_CHECK=1 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-}
fi
if [ "$MODE" = cfg3 ]; then
  step cfg3 900 python -u bench.py --config cfg3 --steps 3 --warmup 1
fi
if [ "$MODE" = spill ]; then
  step spill 700 python -u -m pytest tests/test_spill_gpu.py -v --timeout 650 --timeout-method thread
fi
done
echo ALL DONE
