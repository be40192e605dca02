#!/bin/bash
# per-round evidence (ROUND, default r04): the driver's bench command under rocprofv3 (kernel trace: per-launch
# durations of the timed steps), separate FETCH_SIZE / WRITE_SIZE passes for `traffic`, cfg2 at
# cfg4's 4 KiB-leg size, and the cfg4 line under a kernel trace.  Outputs under
# gpurun_out/${ROUND:-r04}/ev_$TAG/; scripts/summarize_evidence.py turns them into profiles/<round>/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-r04}/ev_${TAG:-run}
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
P="rocprofv3 --output-format csv"
SHORT="--steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-crc --no-ceiling"
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = driver ]; then
  step driver_trace 600 $P --kernel-trace --stats -d $O/driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
  step fetch 240 $P --pmc FETCH_SIZE -d $O/fetch -o run -- python3 bench.py $SHORT
  step write 240 $P --pmc WRITE_SIZE -d $O/write -o run -- python3 bench.py $SHORT
fi
if [ "$MODE" = all ] || [ "$MODE" = cfg4 ]; then
  step cfg2_845k 600 $P --kernel-trace --stats -d $O/cfg2_845k -o run -- python3 bench.py --blocks 845553 --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-crc --no-ceiling
  step cfg4_trace 900 $P --kernel-trace --stats -d $O/cfg4 -o run -- python3 bench.py --config cfg4 --no-cpu-baseline --no-e2e
fi
echo ALL DONE
