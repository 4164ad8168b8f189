"""ASan / UBSan run of the host-side C/C++ (sanitizers): the A*
and OD-bank builder (multi_agent_aac_amd/csrc/aac_host.cpp) and the C oracle with its exact threshold
fallbacks (oracle/aac_oracle.c), driven by tests/sanitize/san_driver.c.  GPU sanitizers are not
available on this pool; the HIP kernels are covered by the compile-time no-scratch guard and the
parity tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not shutil.which("g++") or not shutil.which("make"), reason="no host toolchain")
def test_host_code_is_asan_ubsan_clean():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "san_driver")], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitized run ok" in r.stdout
