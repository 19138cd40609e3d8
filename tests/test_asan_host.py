"""Host code under AddressSanitizer + UBSan (SURVEY.md §5's sanitizer
build, CPU only): `make check-asan` builds host/check_host.cpp with the host
parity layer (host/tsp_host.cpp) and K2's host algorithms
(csrc/search_host.cpp) instrumented, drives them over a grid of sizes and
edge cases, and compares them with the CPU oracle.  Any sanitizer report
aborts the run (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tsp-mpi-reduction_amd")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_check_asan():
    p = subprocess.run(["make", "-s", "-C", PKG, "check-asan"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert "check_host: ok (0 mismatches)" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_xfer_pool_threads_tsan():
    """The small-transfer path's pinned-slot pool (csrc/xfer_pool.h, the code
    xfer.hip runs) driven by eight threads at once under ThreadSanitizer: no
    slot shared, no wait on another stream's event, no wait under the lock
    (round-5 ADVICE on csrc/xfer.hip), no deadlock."""
    p = subprocess.run(["make", "-s", "-C", PKG, "check-xfer"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert "check_xfer: ok" in p.stdout
    assert "ThreadSanitizer" not in p.stderr
