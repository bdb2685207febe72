"""SURVEY §5 sanitizers, on the CPU: the host code that runs concurrently or
hand-counts references, under AddressSanitizer + UBSan and ThreadSanitizer.

* The coalesced drop-in's queue (csrc/pyas_queue.hpp: ring reservation,
  FIFO, caller / dispatcher / completer hand-offs -- the same code
  pyas_coalesce.hip runs) driven by csrc/queue_stress.cpp from 30 caller
  threads, the reference's pool size (active.py:557-589), with a small ring
  so that reservations wrap and wait.  Each caller checks the checksum of
  its own ring bytes; any sanitizer report fails the run.
* The CPython extension (csrc/pyas_fastpath.cpp: manual reference counts on
  its error paths) built with ASan + UBSan, running tests/test_fastpath.py
  with libasan preloaded into the interpreter.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pyactivestorage_amd", "csrc")
SAN = os.path.join(ROOT, "build", "sanitize")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", CSRC, "sanitize", f"SANDIR={SAN}"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return SAN


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_queue_under_sanitizer(built, kind):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(built, f"queue_stress_{kind}"), "30", "300", "65536", "2"],
                       capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "bad 0" in out and "requests 9000" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
    assert "runtime error" not in out


def test_fastpath_under_asan(built):
    import sysconfig
    ext = os.path.join(built, "_fastpath" + sysconfig.get_config_var("EXT_SUFFIX"))
    libasan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    libubsan = subprocess.run(["g++", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    pre = f"{libasan}:{libubsan}"   # the ASan runtime first; anything already preloaded stays
    if os.environ.get("LD_PRELOAD"):
        pre += ":" + os.environ["LD_PRELOAD"]
    env = dict(os.environ, LD_PRELOAD=pre,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_asan_fastpath.py"), ext],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "passed" in out and "failed" not in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
