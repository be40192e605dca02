#!/bin/bash
# profiles/r02 evidence for the decode kernel, before (round-1 final, build/libmtblx_r01.so)
# and after (current): per config (cfg2 4 KiB -> PipeSmall, 64 KiB blocks -> PipeLarge) a
# kernel-trace stats run and separate PMC passes (FETCH_SIZE; WRITE_SIZE; two SQ sets).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r02
mkdir -p $OUT
run() {  # name cmd...
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 240 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for lib in ${LIBS:-cur r01}; do
  LIBARG=""; [ $lib = r01 ] && LIBARG="--lib oxidized-mtbl_amd/build/libmtblx_r01.so"
  for cfg in small large; do
    BA="--no-cpu-baseline --no-e2e --no-crc --no-ceiling $LIBARG"
    [ $cfg = large ] && BA="$BA --block-size 65536 --blocks 6250"
    P="rocprofv3 --output-format csv"
    run ${lib}_${cfg}_stats $P --kernel-trace --stats -d $OUT/${lib}_${cfg}/stats -o run -- python3 bench.py --steps 20 --warmup 5 $BA
    run ${lib}_${cfg}_fetch $P --pmc FETCH_SIZE -d $OUT/${lib}_${cfg}/fetch -o run -- python3 bench.py --steps 3 --warmup 1 $BA
    run ${lib}_${cfg}_write $P --pmc WRITE_SIZE -d $OUT/${lib}_${cfg}/write -o run -- python3 bench.py --steps 3 --warmup 1 $BA
    run ${lib}_${cfg}_sq1 $P --pmc $SQ1 -d $OUT/${lib}_${cfg}/sq1 -o run -- python3 bench.py --steps 3 --warmup 1 $BA
    run ${lib}_${cfg}_sq2 $P --pmc $SQ2 -d $OUT/${lib}_${cfg}/sq2 -o run -- python3 bench.py --steps 3 --warmup 1 $BA
  done
done
echo ALL DONE
