#!/bin/bash
# A/B of snappy library variants (LIBS="name=path ..."): random-byte cfg5 and the compressible stream
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abs
for r in 1 2; do
  for nl in ${LIBS:-cur=}; do
    n=${nl%%=*}; l=${nl#*=}
    for mode in rand comp; do
      X=""; [ $mode = comp ] && X="--compressible --blocks 25000"
      if [ -n "$l" ]; then export MTBLX_LIB=$l; else unset MTBLX_LIB; fi
      timeout -k 10 300 python scripts/snappy_probe.py $X > gpurun_out/abs/${n}_${mode}_$r.log 2>&1 || { tail -3 gpurun_out/abs/${n}_${mode}_$r.log; exit 3; }
      echo "$n $mode $(grep '^decompress' gpurun_out/abs/${n}_${mode}_$r.log | head -1 | cut -c1-120)"
    done
  done
done
