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
  step gpu_tests 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-}
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
if [ "$MODE" = encpmc ]; then   # k_encode traffic: FETCH_SIZE and WRITE_SIZE in separate passes, one cfg3 chunk
  B="python3 bench.py --config cfg3 --cfg3-blocks 100000 --steps 1 --warmup 0"
  step enc_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/enc_trace -o run -- $B
  step enc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_encode --output-format csv -d $O/enc_fetch -o run -- $B
  step enc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_encode --output-format csv -d $O/enc_write -o run -- $B
fi
if [ "$MODE" = fab ]; then   # fused verify A/B: the product vs build/libmtblx_${FV:-fmfma}.so (parity first)
  V=oxidized-mtbl_amd/build/libmtblx_${FV:-fmfma}.so
  step gpu_fab_tests 400 env MTBLX_LIB=$V python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_decode_gpu.py::test_fused_verify_decode tests/test_robust_gpu.py tests/test_writer_gpu.py::test_restart_kat_device
  BB="python bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-ceiling"
  step fab_prod 300 $BB
  step fab_var 300 env MTBLX_AB_CRC=1 $BB --lib $V
  step fab_prod64 300 $BB --block-size 65536 --blocks 6000
  step fab_var64 300 env MTBLX_AB_CRC=1 $BB --block-size 65536 --blocks 6000 --lib $V
  grep -h -o '"decode_blocks_verify".*"vs_decode' $O/fab_*.log || true
fi
if [ "$MODE" = encab ]; then   # k_encode A/B on one cfg3 chunk: product vs build/libmtblx_<v>.so for v in $ENCV
  B="python bench.py --config cfg3 --cfg3-blocks 100000 --steps 1 --warmup 0"
  step encab_prod1 300 $B
  for v in ${ENCV:-}; do step encab_$v 300 $B --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done
  step encab_prod2 300 $B
  grep -h -o '"encode_GiB_per_s": [0-9.]*' $O/encab_*.log || true
fi
if [ "$MODE" = spill ]; then
  step spill 700 python -u -m pytest tests/test_spill_gpu.py -v --timeout 650 --timeout-method thread
fi
done
echo ALL DONE
