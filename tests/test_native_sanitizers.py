"""Race / memory-error detection for the native CPU runtime (host code only).

The reference ships no sanitizer runs; here the thread pool, the
CPU GARs and the pinned mailbox are exercised by a self-test binary compiled with
ThreadSanitizer, AddressSanitizer and UBSan (``garfield_amd/csrc/selftest.cpp``)."""
import os
import shutil
import subprocess

import pytest

from garfield_amd.csrc import build as nb


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("sanitizer", ["thread", "address", "undefined"])
def test_native_selftest_under_sanitizer(sanitizer, tmp_path):
    exe = nb.build_selftest(sanitizer, tmp_path)
    env = dict(os.environ, GARFIELD_NUM_THREADS="8", TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "selftest: ok" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
    assert "runtime error" not in out
