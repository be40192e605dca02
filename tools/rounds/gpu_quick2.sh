#!/bin/bash
# quick check: one test file + bench in driver mode + default + stamps build
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-1500; if [ $rc -ge 124 ]; then exit $rc; fi; }
run t_robust 300 python -u -m pytest tests/test_robust_gpu.py tests/test_cfg4_gpu.py tests/test_reader_gpu.py -x -v --timeout 200 --timeout-method thread
run b_drv 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-e2e --no-cpu-baseline
run b_200 200 python bench.py --steps 200 --warmup 20 --no-e2e --no-cpu-baseline --no-crc
run b_stamps 200 python bench.py --steps 50 --warmup 10 --stamps --no-e2e --no-cpu-baseline --no-ceiling
