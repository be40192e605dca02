"""Kernel resource guard (CPU, hipcc cross-compile): no device kernel may spill to scratch.

The fused-verify decode kernels (k_decode_pipe<PipeSmallV/PipeLargeV>) sit at their 128-VGPR
cap (1024-thread workgroups); a change that added four 16-byte registers to the key copy made
them spill (256-320 B of scratch per lane), and the spilling PipeLargeV then faulted on the GPU
(HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in tests/test_decode_gpu.py::test_fused_verify_decode).
This compiles every .hip source to gfx950 assembly and checks each kernel's
.amdhsa_private_segment_fixed_size, so such a change fails here, before it reaches a GPU.
"""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "oxidized-mtbl_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# kernels allowed a (small, long-standing) private segment: name fragment -> max bytes per lane
ALLOWED = {"k_encode": 32}


def _kernels(path, tmp):
    out = os.path.join(tmp, os.path.basename(path) + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
           "--cuda-device-only", "-S", path, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    text = open(out).read()
    res = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", text, re.S):
        body = m.group(2)
        scratch = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", body).group(1))
        vgpr = int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", body).group(1))
        res[m.group(1)] = (scratch, vgpr)
    return res


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_no_kernel_spills_to_scratch(tmp_path):
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    assert srcs
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        found = {}
        for r in ex.map(lambda p: _kernels(p, str(tmp_path)), srcs):
            found.update(r)
    assert any("k_decode_pipe" in k for k in found), sorted(found)
    bad = []
    for k, (scratch, vgpr) in found.items():
        cap = next((v for frag, v in ALLOWED.items() if frag in k), 0)
        if scratch > cap:
            bad.append((k, scratch, vgpr))
    assert not bad, f"kernels with scratch (name, bytes per lane, vgprs): {bad}"
