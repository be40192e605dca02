#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "crc or verify or robust or reader or pipe" --timeout 240 --timeout-method thread > gpurun_out/crc_tests.log 2>&1; rc=$?
tail -3 gpurun_out/crc_tests.log
[ $rc -eq 0 ] || exit 1
for nl in ${LIBS:-cur=}; do n=${nl%%=*}; l=${nl#*=}; L=""; [ -n "$l" ] && L="--lib $l"; echo "== $n"
MTBLX_AB_CRC=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-ceiling --steps 50 --warmup 10 $L > gpurun_out/crc_bench.log 2>&1 || exit 3
python3 -c "
import json
for l in open('gpurun_out/crc_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('crc32c_verify')))"
done
