"""Kernel resource guard (CPU, hipcc cross-compile): no device kernel may spill to scratch or
make an out-of-line call.

The fused-verify decode kernels (k_decode_pipe<PipeSmallV/PipeLargeV>) sit at their 128-VGPR
cap (1024-thread workgroups). In round 2 a change pushed them over it and PipeLargeV faulted on
the GPU (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in test_fused_verify_decode). Round 3 split
that into its two ingredients:
  * spilling alone is safe: libmtblx_spill.so (-DMTBLX_SPILL, every pipe kernel spills up to
    100 B per lane) passes the whole parity set on the GPU (tests/test_spill_gpu.py);
  * the fault came from the compiler OUTLINING pipe_crc once the kernel ran out of registers:
    build/libmtblx_crcnoinline.so (-DMTBLX_CRC_NOINLINE, pipe_crc a real call, TileArgs and the
    LDS buffer passed as generic pointers) faults in PipeLargeV with no spill pad at all.
The product forces pipe_crc inline. This compiles every .hip source to gfx950 assembly and
checks each kernel's .amdhsa_private_segment_fixed_size (scratch costs bandwidth) and that no
s_swappc (call) is emitted anywhere, so either regression fails here before it reaches a GPU.
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
ALLOWED = {"k_encode": 48}


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
    calls = len(re.findall(r"^\s*s_swappc_b64", text, re.M))
    return res, calls


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_no_kernel_spills_to_scratch(tmp_path):
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    assert srcs
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        found, calls = {}, {}
        for p, (r, c) in zip(srcs, ex.map(lambda p: _kernels(p, str(tmp_path)), srcs)):
            found.update(r)
            calls[os.path.basename(p)] = c
    assert any("k_decode_pipe" in k for k in found), sorted(found)
    bad = []
    for k, (scratch, vgpr) in found.items():
        cap = next((v for frag, v in ALLOWED.items() if frag in k), 0)
        if scratch > cap:
            bad.append((k, scratch, vgpr))
    assert not bad, f"kernels with scratch (name, bytes per lane, vgprs): {bad}"
    assert not any(calls.values()), f"out-of-line device calls per source: {calls}"
