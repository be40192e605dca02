#!/bin/bash
# all GPU tests + bench (driver mode, 200 steps) + stamps timeline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-1200; if [ $rc -ne 0 ]; then exit $rc; fi; }
run tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run b_drv 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-crc
run b_200 200 python bench.py --steps 200 --warmup 20 --no-e2e --no-cpu-baseline --no-crc
run b_stamps 200 python bench.py --steps 50 --warmup 10 --stamps --no-e2e --no-cpu-baseline --no-ceiling
