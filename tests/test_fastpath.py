"""The drop-in's CPython hot path (pyas_fastpath.cpp), on the CPU.

``_fastpath.reduce`` replays a call shape registered by the Python planner
and builds the reference's return objects in C.  Here the coalesced native
call is replaced by a ctypes callback that writes a known partial, so the
key matching and the result objects can be checked without a GPU: they
must be identical to :func:`results.build_one` / :func:`results.build`
(storage.py:98-100 return types).
"""
import ctypes

import numpy as np
import pytest

from pyactivestorage_amd import _lib, results
from pyactivestorage_amd.engine import partial_dtype

_fastpath = pytest.importorskip("pyactivestorage_amd._fastpath")

FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                      ctypes.c_int64, ctypes.POINTER(_lib.Partial), ctypes.POINTER(ctypes.c_int64))
CALLS = []
NEXT = {}


@FN
def _fake(co, path, off, size, desc, mask, sel, pool, pool_len, n_out, out, info):
    CALLS.append((path, off, size, bool(sel)))
    p = NEXT["p"]
    ctypes.memmove(out, p.ctypes.data, 32)
    return NEXT.get("rc", 0)


@pytest.fixture(autouse=True)
def bound():
    _fastpath.clear()
    _fastpath.bind(ctypes.cast(_fake, ctypes.c_void_p).value, 1, np.ma.MaskedArray)
    CALLS.clear()
    yield
    _fastpath.clear()
    _fastpath.bind(0, 0, np.ma.MaskedArray)


def _state(x):
    if isinstance(x, np.ma.MaskedArray):
        d = dict(x.__dict__)
        m = d.pop("_mask")
        return (type(x), x.dtype.str, x.shape, np.asarray(x.data).tobytes(), m is np.ma.nomask,
                np.asarray(m).tobytes(), repr(sorted(d.items(), key=lambda kv: kv[0])))
    return (type(x), x.dtype.str, x.shape, np.asarray(x).tobytes())


def _register(missing, dtype, shape, sel, axis, method, kind, is_ma, has_rule, n_sel, nd=3,
              sel_bytes=None):
    dt = np.dtype(dtype)
    rdt = (np.dtype(np.int64) if dt.kind == "i" else np.dtype(np.uint64) if dt.kind == "u"
           else dt.newbyteorder("=")) if kind == "sum" else dt.newbyteorder("=")
    return _fastpath.register(missing, dtype, None, None, shape, "C", sel, axis, method,
                              bytes(_lib.ChunkDesc()), bytes(_lib.Mask()), sel_bytes, b"", nd,
                              {"sum": 0, "min": 1, "max": 2}[kind], is_ma, has_rule, n_sel,
                              {"f": 0, "i": 1, "u": 2}[dt.kind], rdt.num)


@pytest.mark.parametrize("dtype", ["<f4", ">f8", "<i2", "<u4", "<i8", "u1"])
@pytest.mark.parametrize("kind,method", [("sum", np.ma.sum), ("min", np.ma.min), ("max", np.min)])
def test_replayed_call_builds_the_reference_objects(dtype, kind, method):
    dt = np.dtype(dtype)
    pdt = partial_dtype(dt)
    missing = (dt.type(3), None, None, None)
    shape = (8, 8, 8)
    sel = (slice(0, 8), slice(None), slice(2, 6, 1))
    axis = (0, 1, 2)
    is_ma = method in (np.ma.sum, np.ma.min, np.ma.max)
    assert _register(missing, dt, shape, sel, axis, method, kind, is_ma, True, 256)
    assert _fastpath.size() == 1
    for cnt in (256, 100, 0):
        p = np.zeros(1, dtype=pdt)
        p["count"] = cnt
        p["sum"] = 1e3 + 0.123456789 if dt.kind == "f" else 1000
        p["min"] = 5
        p["max"] = 77
        NEXT["p"] = p
        got = _fastpath.reduce("/tmp/x", 4096, 512, None, None, missing, dt, shape, "C",
                               (slice(0, 8), slice(None), slice(2, 6, 1)), axis, method)
        want = results.build_one(p[0], (1, 1, 1), kind, is_ma, dt, True, 512, 256)
        assert got is not None
        assert _state(got[0]) == _state(want[0]), (cnt, got, want)
        assert _state(got[1]) == _state(want[1])
    assert CALLS[-1] == (b"/tmp/x", 4096, 512, False)


def test_unmasked_plain_method_returns_ndarray():
    dt = np.dtype("<f4")
    missing = (None, None, None, None)
    shape = (4, 4)
    assert _register(missing, dt, shape, (slice(None), slice(None)), (0, 1), np.sum, "sum", False,
                     False, 16, nd=2)
    p = np.zeros(1, dtype=partial_dtype(dt))
    p["count"], p["sum"] = 16, 120.0
    NEXT["p"] = p
    got = _fastpath.reduce("/tmp/x", 0, 64, None, None, missing, dt, shape, "C",
                           (slice(None), slice(None)), (0, 1), np.sum)
    assert type(got[0]) is np.ndarray and got[0].dtype == np.float32 and got[0].shape == (1, 1)
    assert float(got[0][0, 0]) == 120.0 and got[1].dtype == np.int64 and int(got[1][0, 0]) == 16


def test_misses_return_none():
    dt = np.dtype("<f4")
    missing = (np.float32(1), None, None, None)
    shape = (4, 4, 4)
    sel = (slice(0, 4), slice(0, 4), slice(0, 4))
    assert _register(missing, dt, shape, sel, (0, 1, 2), np.ma.sum, "sum", True, True, 64)
    p = np.zeros(1, dtype=partial_dtype(dt))
    NEXT["p"] = p
    args = ["/tmp/x", 0, 256, None, None, missing, dt, shape, "C", sel, (0, 1, 2), np.ma.sum]
    assert _fastpath.reduce(*args) is not None
    # equal-valued dtype objects share the plan (np.dtype keyed by value), and
    # so do equal chunk shapes built per call (a tuple or list of ints)
    assert _fastpath.reduce(*(args[:6] + [np.dtype("float32")] + args[7:])) is not None
    assert _fastpath.reduce(*(args[:7] + [tuple([4, 4, 4])] + args[8:])) is not None
    assert _fastpath.reduce(*(args[:7] + [[4, 4, 4]] + args[8:])) is not None
    for i, other in ((5, (np.float32(1), None, None, None)),     # another missing object
                     (7, (4, 4, 8)),                             # another chunk shape
                     (7, (4, 4)),
                     (7, (np.int64(4), 4, 4)),                   # not plain ints: by identity
                     (9, (slice(0, 4), slice(0, 4), slice(0, 3))),
                     (9, (0, slice(0, 4), slice(0, 4))),         # integer index: not cached
                     (10, [0, 1, 2]),                            # list axis: not cached
                     (10, (0, 1)),
                     (11, np.ma.max),
                     (8, "F"),
                     (6, np.dtype(">f4"))):
        a = list(args)
        a[i] = other
        assert _fastpath.reduce(*a) is None, (i, other)
    NEXT["rc"] = _lib.EIO           # a failed native call falls back (returns None)
    try:
        assert _fastpath.reduce(*args) is None
    finally:
        NEXT.pop("rc")
    assert _fastpath.reduce(b"/tmp/x", 0, 256, *args[3:]) is not None
    assert _fastpath.reduce(12345, 0, 256, *args[3:]) is None      # not a path


def test_register_rejects_bad_shapes():
    dt = np.dtype("<f4")
    m = (None,) * 4
    assert not _fastpath.register(m, dt, None, None, (4,), "C", (slice(None),), None, np.ma.sum,
                                  b"x", bytes(_lib.Mask()), None, b"", 1, 0, True, False, 4, 0, dt.num)
    assert not _fastpath.register(m, dt, None, None, (4,), "C", (slice(None),), None, np.ma.sum,
                                  bytes(_lib.ChunkDesc()), bytes(_lib.Mask()), b"short", b"", 1, 0,
                                  True, False, 4, 0, dt.num)
    assert _fastpath.CHUNK_DESC_SIZE == ctypes.sizeof(_lib.ChunkDesc)
    assert _fastpath.MASK_SIZE == ctypes.sizeof(_lib.Mask)
