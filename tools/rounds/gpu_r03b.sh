#!/bin/bash
# round 3, second GPU session: the fused-CRC ablations (scripts/fused_ab.py), then the new GPU
# tests (keys > 64 KiB in the emitting seek; compressed / decompressed blocks >= 4 GiB).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03/${TAG:-b}
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 "$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = fab ]; then
  step fused_ab 600 python scripts/fused_ab.py ${FAB_LIBS:-prod abcrc1 abcrc2 abcrc3 abcrc4}
fi
if [ "$MODE" = all ] || [ "$MODE" = newtests ]; then
  step newtests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread ${NEWTESTS:-tests/test_seek_gpu.py::test_keys_over_64kib tests/test_big_block_gpu.py}
fi
echo ALL DONE
