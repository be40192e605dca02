#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -s tests/test_big_block_gpu.py tests/test_seek_gpu.py tests/test_reader_gpu.py tests/test_cpp_api.py tests/test_codecs.py -m gpu -x -v --timeout 600 --timeout-method thread 2>&1 | tee gpurun_out/big_tests.log | grep --line-buffered -E "^\[|PASSED|FAILED|Error" ; rc=${PIPESTATUS[0]}
tail -25 gpurun_out/big_tests.log
exit $rc
