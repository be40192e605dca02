"""A build whose decode pipeline kernels spill to scratch must decode exactly like the product.

Round 2 saw HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in test_fused_verify_decode from a
k_decode_pipe<PipeLargeV> variant that spilled 256-320 B per lane.  Legal register
spilling must not fault, so libmtblx_spill.so (make spill: decode.hip with -DMTBLX_SPILL=32,
32 extra VGPRs kept live across the kernel -> every pipeline kernel spills, PipeLargeV ~450 B
per lane) runs the fused-verify and plain decode parity tests in a child process (MTBLX_LIB)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPILL = os.path.join(ROOT, "oxidized-mtbl_amd", "mtblx", "libmtblx_spill.so")


def test_spilling_build_is_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert os.path.exists(SPILL), "build it first: make -C oxidized-mtbl_amd spill"
    env = dict(os.environ, MTBLX_LIB=SPILL)
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "240",
           "--timeout-method", "thread", "-m", "gpu",
           os.path.join(ROOT, "tests", "test_decode_gpu.py") + "::test_fused_verify_decode",
           os.path.join(ROOT, "tests", "test_decode_gpu.py") + "::test_cfg2_sample_vs_oracle",
           os.path.join(ROOT, "tests", "test_decode_gpu.py") + "::test_mutated_blocks",
           os.path.join(ROOT, "tests", "test_decode_gpu.py") + "::test_64k_blocks_long_keys",
           os.path.join(ROOT, "tests", "test_decode_gpu.py") + "::test_key_tails_dense_and_planes",
           os.path.join(ROOT, "tests", "test_decode_gpu.py") + "::test_directory_in_any_order",
           os.path.join(ROOT, "tests", "test_cfg4_gpu.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
