#!/bin/bash
# A/B/C... on one box: alternating bench runs of several libmtblx builds (LIBS="name=path ...").
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BA="--no-cpu-baseline --no-e2e --no-crc --no-ceiling --steps ${STEPS:-200} --warmup 20 ${BENCH_ARGS:-}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for nv in $LIBS; do
    n=${nv%%=*}; p=${nv#*=}
    timeout -k 10 300 python bench.py $BA --lib $p > gpurun_out/abn_${n}_$r.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/abn_${n}_$r.log; exit 3; }
    python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/abn_${n}_$r.log $n
  done
done
