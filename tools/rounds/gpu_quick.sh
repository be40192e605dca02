#!/bin/bash
# quick iteration: parity tests, bench (no CPU baseline), stamps breakdown
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local n=$1 to=$2; shift 2; echo "=== $n"; timeout -k 10 "$to" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "gpurun_out/$n.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gpu_tests 600 python -m pytest tests -m gpu -x -q
run bench 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-}
run stamps 300 python bench.py --no-cpu-baseline --stamps ${BENCH_ARGS:-}
