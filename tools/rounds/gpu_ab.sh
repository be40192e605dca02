#!/bin/bash
# A/B of decode library variants (LIBS="name=path ..."; "cur" = the product build) on cfg2
# (PipeSmall) and 64 KiB blocks (PipeLarge) [CFGS="small large cfg3"], two rounds, 200 steps each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
val() { python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d.get('ms_per_step'), (d.get('roofline') or {}).get('frac'))" "$1" "$2"; }
BA="--no-cpu-baseline --no-e2e --no-crc --no-ceiling --steps ${STEPS:-200} --warmup 20"
for r in 1 2; do
  for cfg in ${CFGS:-small large}; do
    X=""; [ $cfg = large ] && X="--block-size 65536 --blocks 6250"
    [ $cfg = cfg3 ] && X="--config cfg3 --cfg3-blocks 200000"
    for nl in ${LIBS:-cur=}; do
      n=${nl%%=*}; l=${nl#*=}
      L=""; [ -n "$l" ] && L="--lib $l"
      timeout -k 10 300 python bench.py $BA $X $L > gpurun_out/ab/${n}_$cfg$r.log 2>&1 || { tail -3 gpurun_out/ab/${n}_$cfg$r.log; exit 3; }
      val gpurun_out/ab/${n}_$cfg$r.log ${n}_$cfg
    done
  done
done
