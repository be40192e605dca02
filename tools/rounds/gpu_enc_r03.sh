#!/bin/bash
# Round 3 encode: gather-path parity (encode / writer tests), A/B vs the LDS-assembly build on
# cfg3 chunks, then the CRC kernel A/B.  Outputs under gpurun_out/r03/enc_$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03/enc_${TAG:-run}
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 "$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step t_enc 500 python -u -m pytest tests/test_encode_gpu.py tests/test_writer_gpu.py -x -v --timeout 240 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = ab ]; then
  for r in 1 2; do
    for nl in ${LIBS:-cur= old=oxidized-mtbl_amd/build/libmtblx_encold.so}; do
      n=${nl%%=*}; l=${nl#*=}
      L=""; [ -n "$l" ] && L="--lib $l"
      step ab_${n}_$r 300 python bench.py --config cfg3 --cfg3-blocks ${BLOCKS:-200000} --no-cpu-baseline $L
    done
  done
  for f in $O/ab_*.log; do python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[1], 'enc', d['encode_GiB_per_s'], 'dec', d['value'])" $f; done
fi
if [ "$MODE" = all ] || [ "$MODE" = crc ]; then
  step crc_ab 600 python scripts/crc_ab.py 0 3 5 6
fi
echo ALL DONE
