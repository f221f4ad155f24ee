"""The engine's host-only pieces under AddressSanitizer + UndefinedBehaviorSanitizer (a sanitizer build of
the host C++), no GPU: globalign_amd/csrc/ga_host_selftest.cpp checks the tie-break table (ga_rng.h: the four-word
scan, the resumable stream, the state after D dispatches) against a draw-by-draw restatement of
CPython's random.choice, and the problem checks (ga_check.h: validation, the int32 range guard, word widths).  The same
binary without sanitizers must pass too."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

CSRC = os.path.join(ROOT, "globalign_amd", "csrc")
LIB = os.path.join(ROOT, "globalign_amd", "_lib")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", CSRC, "selftest", "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return True


@pytest.mark.parametrize("binary", ["ga_host_selftest_asan", "ga_host_selftest"])
def test_host_selftest(built, binary):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(LIB, binary)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "all checks passed" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr and "ThreadSanitizer" not in r.stderr
