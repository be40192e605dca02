#!/bin/bash
# Round 4 GPU session: tests (the spilling-build check last), smoke, the driver's bench line.
# Outputs under gpurun_out/r04/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04/${TAG:-run}
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
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
fi
if [ "$MODE" = all ] || [ "$MODE" = crc ]; then
  step crc_ab 600 python scripts/crc_ab.py mfma lanes
fi
if [ "$MODE" = all ] || [ "$MODE" = spill ]; then
  step spill 700 python -u -m pytest tests/test_spill_gpu.py -v --timeout 650 --timeout-method thread
fi
if [ "$MODE" = noinline ]; then   # diagnostic, may fault: always the last step of a call
  step noinline 300 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_crcnoinline.so python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_decode_gpu.py::test_fused_verify_decode
fi
echo ALL DONE
