"""Host-code sanitizers (SURVEY §5 "race detection / sanitizers"): the threaded generators, the
parallel CSR build, the loaders / sidecar cache and the query-parallel CPU BFS, built with
AddressSanitizer + UBSan and with ThreadSanitizer (csrc/Makefile targets asan / tsan, driver
csrc/tests/host_selftest.cpp). GPU ASan is not available on the target pool, so device code is
covered by the deterministic-result GPU tests instead."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "build", "san")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_sanitizer_selftest(tmp_path, kind):
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "csrc"), kind], capture_output=True,
                       text=True, timeout=600)
    if b.returncode != 0:
        pytest.skip(f"{kind} build unavailable: {b.stderr[-400:]}")
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    r = subprocess.run([os.path.join(SAN, f"host_selftest_{kind}"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host selftest: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
