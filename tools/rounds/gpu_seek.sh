#!/bin/bash
# GPU tests touching the reader surfaces (seek-based iteration, device Reader, codecs)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_seek_gpu.py tests/test_reader_gpu.py tests/test_codecs.py tests/test_cpp_api.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > gpurun_out/seek_tests.log 2>&1; rc=$?
tail -25 gpurun_out/seek_tests.log
exit $rc
