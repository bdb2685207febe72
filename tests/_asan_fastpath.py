"""Run tests/test_fastpath.py against the ASan+UBSan build of _fastpath
(build/sanitize, ``make -C pyactivestorage_amd/csrc sanitize``); started
by tests/test_sanitizers.py with libasan preloaded into the interpreter."""
import importlib.machinery
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pyactivestorage_amd  # noqa: E402

path = sys.argv[1]
loader = importlib.machinery.ExtensionFileLoader("pyactivestorage_amd._fastpath", path)
spec = importlib.util.spec_from_file_location("pyactivestorage_amd._fastpath", path, loader=loader)
mod = importlib.util.module_from_spec(spec)
loader.exec_module(mod)
sys.modules["pyactivestorage_amd._fastpath"] = mod
pyactivestorage_amd._fastpath = mod
assert mod.__file__ == path

import pytest  # noqa: E402

sys.exit(pytest.main(["-q", "-p", "no:cacheprovider", os.path.join(ROOT, "tests", "test_fastpath.py")]))
