set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do for nv in base=oxidized-mtbl_amd/build/libmtblx_encbase.so new=oxidized-mtbl_amd/mtblx/libmtblx.so; do
  n=${nv%%=*}; p=${nv#*=}
  timeout -k 10 300 python bench.py --config cfg3 --cfg3-blocks 100000 --cfg3-chunk 100000 --no-cpu-baseline --lib $p > gpurun_out/enc_${n}_$r.log 2>&1 || { echo FAIL; tail -5 gpurun_out/enc_${n}_$r.log; exit 3; }
  python3 -c "import sys,json
for l in open(sys.argv[1]):
  if l.startswith('{'):
    d=json.loads(l); print(sys.argv[2], d['value'], d['encode_GiB_per_s'], d['roofline'].get('encode') if 'roofline' in d else '')" gpurun_out/enc_${n}_$r.log $n
done; done
