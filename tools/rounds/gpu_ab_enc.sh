#!/bin/bash
# A/B of encode library variants on one cfg3 chunk (LIBS="name=path ..."; "cur" = the product build)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abe
for r in 1 2; do
  for nl in ${LIBS:-cur=}; do
    n=${nl%%=*}; l=${nl#*=}
    L=""; [ -n "$l" ] && L="--lib $l"
    timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks ${BLOCKS:-200000} --no-cpu-baseline $L > gpurun_out/abe/${n}_$r.log 2>&1 || { tail -3 gpurun_out/abe/${n}_$r.log; exit 3; }
    python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], 'enc', d['encode_GiB_per_s'], 'dec', d['value'], 'mismatch', d.get('mismatches'))" gpurun_out/abe/${n}_$r.log $n
  done
done
