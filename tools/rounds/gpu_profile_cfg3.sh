#!/bin/bash
# k_decode_pipe<PipeLarge> and k_encode on one cfg3 chunk (100 000 x 64 KiB blocks, Zipf keys):
# kernel-trace stats and separate PMC passes (FETCH_SIZE; WRITE_SIZE; SQ), each its own run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_cfg3
mkdir -p $OUT
B="python3 bench.py --config cfg3 --cfg3-blocks 100000 --cfg3-chunk 100000 --no-cpu-baseline"
P="rocprofv3 --output-format csv"
run() {  # name cmd...
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
run stats $P --kernel-trace --stats -d $OUT/stats -o run -- $B
run fetch $P --pmc FETCH_SIZE -d $OUT/fetch -o run -- $B
run write $P --pmc WRITE_SIZE -d $OUT/write -o run -- $B
run sq $P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/sq -o run -- $B
echo ALL DONE
