"""CPU: the oracle (the CPU restatement every GPU result is checked against)
under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer, as
SURVEY.md section 5 plans ("a CPU restatement under -fsanitize=thread,address").
oracle/san_driver.cc drives every oracle entry point over one synthetic batch,
including the rwlock Procs of the multi-core baseline (fuzzer.go:494-511)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def san_build():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "san"], capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "fsanitize" in r.stderr and "cannot find" in r.stderr:
        pytest.skip("sanitizer runtimes are not installed: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(ORACLE, "_san")


@pytest.mark.parametrize("kind,args", [("asan", ["48", "8"]), ("tsan", ["48", "8"]), ("tsan", ["16", "3"])])
def test_oracle_under_sanitizer(san_build, kind, args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(san_build, "driver_" + kind)] + args, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "0 failures" in r.stdout
