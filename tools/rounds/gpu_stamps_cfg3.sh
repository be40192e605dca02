set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/st
for n in ${STN:-stL stE}; do
  timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks 100000 --no-cpu-baseline --no-get --stamps --lib oxidized-mtbl_amd/build/libmtblx_$n.so > gpurun_out/st/$n.log 2>&1 || { tail -5 gpurun_out/st/$n.log; exit 3; }
  python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], json.dumps(d.get('phase_cycles_per_tile')))" gpurun_out/st/$n.log $n
done
