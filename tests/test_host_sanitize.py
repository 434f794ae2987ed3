"""Host C++ of the library (kf_host.cpp: vocab tables, record index, `.kf`
formatter and threaded writer) under AddressSanitizer + UBSan:
`python -m kf2vecfsw_amd.build --sanitize` builds tests/host_sanitize.cpp with
kf_host.cpp and runs it; any sanitizer report aborts with a non-zero status."""
import os
import subprocess


def test_host_code_clean_under_asan_ubsan():
    from kf2vecfsw_amd import build as B
    exe = B.build_sanitized_host()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
