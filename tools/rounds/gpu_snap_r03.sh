#!/bin/bash
# Round 3 device snappy: k_snappy_lanes parity (snappy tests under auto and lanes-only routing),
# then compressible / random timings per routing.  Outputs under gpurun_out/r03/snap_$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03/snap_${TAG:-run}
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
step t_auto 400 $T tests/test_snappy_gpu.py tests/test_pipe_gpu.py
step t_lanes 400 env MTBLX_SNAPPY_KERNEL=lanes $T tests/test_snappy_gpu.py

for m in ${MODES:-quads lanes auto}; do
  step p_comp_$m 300 env MTBLX_SNAPPY_KERNEL=$m python scripts/snappy_probe.py --compressible --blocks 100000 --tile 4
  step p_rand_$m 300 env MTBLX_SNAPPY_KERNEL=$m python scripts/snappy_probe.py --blocks 100000
done
for f in $O/p_*.log; do echo "$f $(grep decompress $f)"; done
echo ALL DONE
