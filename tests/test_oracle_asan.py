"""The oracle's known-answer tests again, against the AddressSanitizer + UndefinedBehaviorSanitizer build of the same C
sources (oracle/Makefile `asan`), in a child process with libasan preloaded: memory errors or UB in the checker would
otherwise pass silently. Host code only (no GPU)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    cc = shutil.which("gcc")
    if not cc:
        return None
    p = subprocess.run([cc, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_kats_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc's libasan is not available")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ, EKO_LIB=os.path.join(ROOT, "oracle", "libekoracle_asan.so"), LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(ROOT, "tests", "test_oracle_kat.py"),
                        os.path.join(ROOT, "tests", "test_incremental_oracle.py"),
                        os.path.join(ROOT, "tests", "test_hopping_gap.py")],
                       env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed" in r.stdout
