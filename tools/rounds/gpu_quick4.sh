#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600; if [ $rc -ge 124 ]; then exit $rc; fi; }
run t_writer 300 python -u -m pytest tests/test_writer_gpu.py -x -v --timeout 200 --timeout-method thread
run b_stamps 200 python bench.py --steps 50 --warmup 10 --stamps --no-e2e --no-cpu-baseline --no-ceiling
