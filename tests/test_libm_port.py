"""The device's logf/expf (slam-maskrcnn_amd/csrc/semtsdf_libm.h) equal the host C library's
bit for bit over the association's whole input domain (CPU half; the device half is
tests/test_gpu_assoc_exact.py).  The reference's filter_overlaps (src/SfM_CUDA/tsdf.cu:
318,329,343) calls logf/expf on the host; glibc's are not correctly rounded, so the device's
exact association path must reproduce them rather than compute its own."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "helpers", "libm_port_check.cpp")


def _fma_host() -> bool:
    with open("/proc/cpuinfo") as f:
        flags = f.read()
    return " fma " in flags and " avx2 " in flags


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_libm_port_equals_host_libm_exhaustively():
    if not _fma_host():
        pytest.skip("host libm selects its non-FMA variant on this CPU (the port restates the FMA one)")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "chk")
        subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-o", exe, SRC, "-lm"])
        out = subprocess.run([exe, "0.05", "1"], capture_output=True, text=True, check=True, timeout=600).stdout
    res = {ln.split()[0]: (int(ln.split()[1]), int(ln.split()[2])) for ln in out.splitlines()}
    assert res["logf"][0] > 36_000_000 and res["logf"][1] == 0, res
    assert res["expf"][0] > 1_000_000_000 and res["expf"][1] == 0, res
    assert res["spot"][1] == 0, res
