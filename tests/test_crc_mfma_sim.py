"""CPU check of the matrix-core CRC-32C's constant operands (csrc/crc_mfma.h): tests/cpp/
crc_mfma_sim.cpp evaluates every MFMA of k_crc32c_mfma as sums over lane groups and operand
slots, with the operands filled as the kernel fills them, and compares with a bytewise
CRC-32C (crate crc32c 0.4's checksum, /root/reference/src/reader.rs:159-164) on every length
4..2100 at all alignments and on blocks of several super-windows.  The GPU run of the same
kernel is tests/test_crc_mfma_gpu.py."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not present")
def test_crc_mfma_tables_model(tmp_path):
    exe = tmp_path / "crc_mfma_sim"
    r = subprocess.run([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                        "-I" + os.path.join(ROOT, "oxidized-mtbl_amd", "csrc"),
                        os.path.join(ROOT, "tests", "cpp", "crc_mfma_sim.cpp"), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr
