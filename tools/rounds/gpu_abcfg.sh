#!/bin/bash
# A/B of several libmtblx builds (LIBS="name=path ...") on cfg2 (default bench), a 100k-block
# cfg3 round trip and a 1 GiB cfg4 (device-resident legs); one line per run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for nv in $LIBS; do
    n=${nv%%=*}; p=${nv#*=}
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-crc --no-ceiling --steps 100 --warmup 10 --lib $p > gpurun_out/abc2_${n}_$r.log 2>&1 || { echo "FAIL cfg2 $n"; exit 3; }
    timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks 100000 --cfg3-chunk 100000 --no-cpu-baseline --lib $p > gpurun_out/abc3_${n}_$r.log 2>&1 || { echo "FAIL cfg3 $n"; exit 3; }
    python3 -c "import sys,json
v=[]
for f in sys.argv[2:]:
  for l in open(f):
    if l.startswith('{'):
      d=json.loads(l); v.append(d['value'])
print(sys.argv[1], *v)" $n gpurun_out/abc2_${n}_$r.log gpurun_out/abc3_${n}_$r.log
  done
done
