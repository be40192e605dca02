#!/bin/bash
# parity tests + bench + stamps for the product build and the ablation builds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local n=$1 to=$2; shift 2; echo "=== $n"; timeout -k 10 "$to" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -1 "gpurun_out/$n.log" | python3 -c "import sys,json
l=sys.stdin.read().strip()
try:
  d=json.loads(l); print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac']); print(d.get('phase_cycles_per_tile'))
except Exception: print(l[-300:])"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then run gpu_tests 600 python -m pytest tests -m gpu -x -q; tail -2 gpurun_out/gpu_tests.log; grep -q " passed" gpurun_out/gpu_tests.log && ! grep -q "failed" gpurun_out/gpu_tests.log || { echo "TESTS FAILED: stop"; exit 1; }; fi
run bench 300 python bench.py --no-cpu-baseline
run stamps 300 python bench.py --no-cpu-baseline --stamps
for v in ${ABL:-nokey noval nocopy}; do
  run abl_$v 300 python bench.py --no-cpu-baseline --stamps --lib oxidized-mtbl_amd/build/libmtblx_$v.so
done
