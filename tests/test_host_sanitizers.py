"""Host runtime under sanitizers: the C++ self-test
(csrc/tests/host_selftest.cc -- tracker, sliding window, shared-memory control
queue with 4 producer threads, CSV parser, CSV logger + metrics sink with an
asynchronous producer) built with ASAN+UBSAN and with TSAN, run on the CPU.
GPU-side sanitizers are not available on this pool."""
import os
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "csrc"))


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_host_selftest_sanitized(san):
    import build

    exe = build.build_selftest(san)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["TSAN_OPTIONS"] = "halt_on_error=1:second_deadlock_stack=1"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
