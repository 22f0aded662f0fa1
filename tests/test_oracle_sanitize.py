"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host code only): the
oracle golden and property suites rerun in a child process against liboracle_san.so
(ORACLE_SANITIZE=1) with libasan preloaded; any out-of-bounds access, use after free,
signed overflow, bad shift or misaligned access aborts the child."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _runtime(name):
    try:
        path = subprocess.check_output(["gcc", f"-print-file-name={name}"], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_suites_under_asan_ubsan():
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("gcc's libasan runtime is not installed")
    env = dict(os.environ, ORACLE_SANITIZE="1", LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("PYTEST_ADDOPTS", None)
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
           os.path.join(ROOT, "tests", "test_oracle_golden.py"), os.path.join(ROOT, "tests", "test_oracle_props.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
