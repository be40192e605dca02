#!/bin/bash
# Evidence session for the round: GPU parity tests -> full bench (with cpu_baseline) ->
# rocprofv3 kernel-trace stats -> two separate PMC passes (FETCH_SIZE, WRITE_SIZE; the TCC
# block cannot hold both, MI355X_MICROARCH.md "rocprofv3 PMC slots").  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 50 --warmup 10
rm -rf gpurun_out/prof_$TAG
step prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e
step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$TAG/fetch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-crc
step prof_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$TAG/write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-crc
find gpurun_out/prof_$TAG -name "*.csv" | sort
