"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer and
under ThreadSanitizer (sanitizer runs of the CPU path): builds
`make -C oracle asan tsan` and runs oracle/sanitize_main.c, which drives
every oracle entry point -- the batched solve on a 4-thread pool with and
without margins, a single solve with tables and gate margin, the Hungarian
comparator -- and checks that every output is a permutation."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_oracle_under_sanitizer(kind):
    b = subprocess.run(["make", "-C", ORACLE, kind], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    r = subprocess.run([os.path.join(ORACLE, "_san", "oracle_" + kind)], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize driver: ok" in r.stdout
    assert "runtime error" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
