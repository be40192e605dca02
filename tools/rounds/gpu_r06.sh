#!/bin/bash
# Round 6 GPU session: MODES = tests | smoke | bench | cfg3 | cfg3oracle | bounds | ... (space separated).
# Outputs under gpurun_out/r06/<TAG>/.  Every GPU step has its own time limit; a step that
# times out, aborts or faults ends the call (test failures, rc 1, of a gpu_* step do not).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/${TAG:-run}
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
PT="python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
for MODE in ${MODES:-tests smoke bench}; do
case $MODE in
tests) step gpu_tests 1000 $PT tests -m gpu --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-} ;;
sel) step gpu_sel 600 $PT ${SEL} ;;
smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
bench) step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
cfg3) step cfg3 900 python -u bench.py --config cfg3 --steps 3 --warmup 1 ;;
cfg3oracle)   # every cfg3 block against the oracle, full size (1 M blocks, 10 chunks)
  rm -f $O/cfg3_oracle.txt
  step gpu_cfg3_oracle 1100 env MTBLX_CFG3_BLOCKS=${CFG3_BLOCKS:-1000000} MTBLX_CFG3_LOG=$O/cfg3_oracle.txt \
    python -u -m pytest -v -s --timeout 1050 --timeout-method thread -p no:cacheprovider tests/test_cfg3_oracle_gpu.py ;;
poison) step gpu_poison 1100 env MTBLX_POISON=1 $PT tests -m gpu --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-} ;;
bounds) step gpu_bounds 1150 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_bounds.so MTBLX_BOUNDS_CHECK=1 $PT tests -m gpu --deselect tests/test_spill_gpu.py::test_spilling_build_is_exact ${PYTEST_ARGS:-} ;;
encab)   # k_encode A/B on one cfg3 chunk: product vs build/libmtblx_<v>.so for v in $ENCV, twice
  B="python bench.py --config cfg3 --cfg3-blocks 100000 --steps 1 --warmup 0 --no-cpu-baseline"
  for r in 1 2; do
    step encab_prod$r 300 $B
    for v in ${ENCV:-}; do step encab_${v}_$r 300 $B --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done
  done
  grep -H -o '"encode_GiB_per_s": [0-9.]*' $O/encab_*.log || true ;;
crcab)   # CRC kernel variants: parity of each (test_crc_mfma_gpu) then scripts/crc_ab.py over all of them
  ARGS=""
  for v in ${CRCV:-}; do
    step gpu_crc_$v 300 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_$v.so $PT tests/test_crc_mfma_gpu.py
    ARGS="$ARGS mfma@oxidized-mtbl_amd/build/libmtblx_$v.so"
  done
  step crcab 600 python -u scripts/crc_ab.py $ARGS ;;
snapprof)   # k_snappy_lanes on the compressible 100 000-block stream: kernel stats + SQ counters (separate passes)
  A="scripts/snappy_probe.py --blocks 100000 --tile 4 --compressible --reps 3"; export MTBLX_SNAPPY_KERNEL=lanes
  P="rocprofv3 --output-format csv"
  step snap_stats 240 $P --kernel-trace --stats -d $O/snap_stats -o run -- python3 $A
  step snap_p1 120 $P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex k_snappy -d $O/snap_p1 -o run -- python3 $A
  step snap_p2 120 $P --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-include-regex k_snappy -d $O/snap_p2 -o run -- python3 $A ;;
snapstat)   # kernel stats of one snappy routing on the compressible stream
  step snapstat 240 env MTBLX_SNAPPY_KERNEL=${SNAPK:-waves} rocprofv3 --kernel-trace --stats --output-format csv -d $O/snapstat -o run -- python3 scripts/snappy_probe.py --blocks 100000 --tile 4 --compressible --reps 3 ;;
snapst)   # k_snappy_waves per-phase stamps (snapstamps diagnostic build)
  step snapst 200 env MTBLX_LIB=oxidized-mtbl_amd/mtblx/libmtblx_snapstamps.so MTBLX_SNAPPY_KERNEL=waves python3 scripts/snappy_probe.py --blocks 100000 --tile 4 --compressible --reps 3 ;;
snapab)   # device snappy kernels on the compressible 100 000-block stream, alternating, HIP events
  for r in 1 2; do
    for k in ${SNAPK:-lanes waves}; do
      step snapab_${k}_$r 200 env MTBLX_SNAPPY_KERNEL=$k python3 scripts/snappy_probe.py --blocks 100000 --tile 4 --compressible --reps 10
    done
  done
  grep -H "decompress" $O/snapab_*.log || true ;;
decab)   # PipeLarge A/B on one cfg3 chunk (decode GiB/s = value): product vs build/libmtblx_<v>.so for v in $DECV, twice
  B="python bench.py --config cfg3 --cfg3-blocks 100000 --steps 3 --warmup 1 --no-cpu-baseline --no-get"
  for r in 1 2; do
    step decab_prod$r 300 $B
    for v in ${DECV:-}; do step decab_${v}_$r 300 $B --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done
  done
  grep -H -o '"value": [0-9.]*' $O/decab_*.log || true ;;
decst)   # PipeLarge per-phase stamps: the product stamps build vs build/libmtblx_<v>.so for v in $STV
  B="python bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline --no-get --stamps"
  step decst_prod 300 $B --lib oxidized-mtbl_amd/mtblx/libmtblx_stamps.so
  for v in ${STV:-}; do step decst_$v 300 $B --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done ;;
encpmc)   # k_encode LDS / wait counters (one PMC pass each): product vs build/libmtblx_<v>.so for v in $ENCV
  A="bench.py --config cfg3 --cfg3-blocks 100000 --steps 1 --warmup 0 --no-cpu-baseline --no-get"
  for v in prod ${ENCV:-}; do
    L=""; [ "$v" = prod ] || L="--lib oxidized-mtbl_amd/build/libmtblx_$v.so"
    step encpmc_$v 200 rocprofv3 --output-format csv --kernel-include-regex k_encode --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS -d $O/encpmc_$v -o run -- python3 $A $L
  done ;;
planab)   # block-cut A/B on three cfg3 chunks (writer_GiB_per_s, plan_ms_total): product vs build/libmtblx_<v>.so for v in $PLANV
  B="python bench.py --config cfg3 --cfg3-blocks 300000 --steps 1 --warmup 0 --no-cpu-baseline --no-get"
  for r in 1 2; do
    step planab_prod$r 300 $B
    for v in ${PLANV:-}; do step planab_${v}_$r 300 $B --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done
  done
  grep -H -o '"plan_ms_total": [0-9.]*\|"writer_GiB_per_s": [0-9.]*' $O/planab_*.log || true ;;
planprof)   # block-cut kernel breakdown: one cfg3 chunk (65 930 240 records, 64 shards), kernel trace
  step planprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/planprof -o run -- python3 scripts/plan_probe.py 65930240 64 ;;
cfg2ab)   # cfg2 decode A/B (bench value, 100 steps): product vs build/libmtblx_<v>.so for v in $DECV, twice; cfg4 legs with $CFG4=1
  B="python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-e2e --no-get --no-ceiling"
  for r in 1 2; do
    step cfg2ab_prod$r 300 $B
    for v in ${DECV:-}; do step cfg2ab_${v}_$r 300 $B --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done
  done
  if [ "${CFG4:-0}" = 1 ]; then
    step cfg4ab_prod 600 python bench.py --config cfg4 --no-cpu-baseline --no-e2e
    for v in ${DECV:-}; do step cfg4ab_$v 600 python bench.py --config cfg4 --no-cpu-baseline --no-e2e --lib oxidized-mtbl_amd/build/libmtblx_$v.so; done
  fi
  grep -H -o '"value": [0-9.]*' $O/cfg2ab_*.log $O/cfg4ab_*.log 2>/dev/null || true ;;
snaplib)   # device snappy (lanes routing) A/B across libraries: product vs build/libmtblx_<v>.so for v in $SNAPV, twice
  for r in 1 2; do
    step snaplib_prod_$r 200 env MTBLX_SNAPPY_KERNEL=lanes python3 scripts/snappy_probe.py --blocks 100000 --tile 4 --compressible --reps 10
    for v in ${SNAPV:-}; do step snaplib_${v}_$r 200 env MTBLX_LIB=oxidized-mtbl_amd/build/libmtblx_$v.so MTBLX_SNAPPY_KERNEL=lanes python3 scripts/snappy_probe.py --blocks 100000 --tile 4 --compressible --reps 10; done
  done
  grep -H "decompress" $O/snaplib_*.log || true ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
done
echo "=== done"
