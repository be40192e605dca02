#!/bin/bash
# Device decode time vs batch size (cfg2 blocks): separates the per-tile cost from the
# launch's fixed cost (pipeline fill/drain, tail imbalance, launch overhead).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BA="--no-cpu-baseline --no-e2e --no-crc --no-ceiling --steps 100 --warmup 10 ${BENCH_ARGS:-}"
for n in ${SIZES:-12288 25000 50000 100000 200000 400000}; do
  timeout -k 10 300 python bench.py $BA --blocks $n > gpurun_out/sz_$n.log 2>&1 || exit 3
  python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['ms_per_step'], list(d['kernels_ms'].values())[0])" gpurun_out/sz_$n.log $n
done
