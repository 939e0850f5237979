"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the CPU code
(VERDICT r1 "next" #8): the oracle restatement and the
library's host C++ (exact table builders incl. the closed-form rank prefix,
count files, argument validation) built with host-only sanitizers by
tests/sanitize/Makefile and run on random inputs.  Any report aborts the
driver (halt_on_error), failing the test."""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-j8", "-C", HERE], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(HERE, "build")


@pytest.mark.parametrize("driver", ["oracle_san", "host_san"])
def test_sanitized_driver(built, driver, tmp_path):
    r = subprocess.run([os.path.join(built, driver)], capture_output=True, text=True, timeout=600, env=ENV,
                       cwd=tmp_path)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "sanitizer run ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
