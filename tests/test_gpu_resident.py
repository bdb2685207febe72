"""Resident mode: ``Active(..., resident=True)`` keeps a variable's decoded
chunks in HBM across queries.  Every query must return exactly what the
non-resident path returns (which the other GPU tests pin to the reference),
while reading from the file only chunks no earlier query loaded.  Covers an
uncompressed variable and the reference's test1.nc (shuffle + zlib, f8).
"""
import numpy as np
import pytest

from pyactivestorage_amd.active import Active, release_resident
from tests import _dist_active as D
from tests.test_gpu_active import variable

pytestmark = pytest.mark.gpu


def _same(a, b, what, method="min"):
    """Bit-exact, except sums/means of shuffled variables: the resident
    store keeps chunks un-shuffled, and the fresh path's fused un-shuffle
    adds the elements in another order (1e-6 relative, the north star's
    tolerance; counts, masks, min and max stay exact)."""
    assert type(a) is type(b) and np.shape(a) == np.shape(b), what
    np.testing.assert_array_equal(np.ma.getmaskarray(a), np.ma.getmaskarray(b), err_msg=what)
    if method in ("sum", "mean"):
        np.testing.assert_allclose(np.ma.getdata(a), np.ma.getdata(b), rtol=1e-6, err_msg=what)
    else:
        np.testing.assert_array_equal(np.ma.getdata(a), np.ma.getdata(b), err_msg=what)


def _query(var, method, axis, index, resident):
    act = Active(var, resident=resident)
    getattr(act, method)(axis=axis)
    r = act[index]
    return r, act.data_read


@pytest.mark.parametrize("make", ["synthetic", "test1.nc:tas"])
def test_resident_matches_fresh(gpu, make):
    var = D.make_variable() if make == "synthetic" else variable(make)
    nd = len(var.shape)
    half = tuple(slice(0, max(1, n // 2)) for n in var.shape)
    other = tuple(slice(n // 3, n) for n in var.shape)
    queries = [("mean", None, half), ("max", (0,), other), ("min", (nd - 1,), (slice(None),) * nd),
               ("mean", (0, nd - 1), half)]
    try:
        seen = 0
        for k, (method, axis, index) in enumerate(queries):
            want, _ = _query(var, method, axis, index, False)
            got, read = _query(var, method, axis, index, True)
            _same(got, want, f"{make} query {k}", method if make != "synthetic" else "exact")
            seen += read
        # every chunk is now resident: a repeat reads nothing
        got, read = _query(var, "mean", None, (slice(None),) * nd, True)
        assert read == 0
        want, full_read = _query(var, "mean", None, (slice(None),) * nd, False)
        _same(got, want, f"{make} repeat", "mean" if make != "synthetic" else "exact")
        assert 0 < seen <= full_read
    finally:
        release_resident(var)
    assert getattr(var, "_pyas_resident", None) is None


def test_resident_concurrent_threads(gpu):
    """Threads share one resident store (the reference drives Active from
    dask worker threads, dask-demo/demo.py:107-168): each thread's queries,
    on its own stream, must see complete chunks."""
    import concurrent.futures
    var = D.make_variable()
    nd = len(var.shape)
    index_list = [tuple(slice(k, n) for n in var.shape) for k in range(8)]
    want = [_query(var, "mean", (0,), ix, False)[0] for ix in index_list]
    try:
        with concurrent.futures.ThreadPoolExecutor(max_workers=8) as ex:
            for rep in range(3):
                got = list(ex.map(lambda ix: _query(var, "mean", (0,), ix, True)[0], index_list))
                for k, (g, w) in enumerate(zip(got, want)):
                    _same(g, w, f"rep {rep} thread query {k}")
    finally:
        release_resident(var)
    assert nd == 3


def test_release_while_queries_run(gpu):
    """release_resident must not free HBM another thread's query
    is reading, and two threads loading the same chunks must not both read
    them: queries racing a release still return the fresh path's answer,
    and the copy is gone once they finish."""
    import concurrent.futures
    import threading
    var = D.make_variable()
    ix = tuple(slice(None) for _ in var.shape)
    want = _query(var, "mean", (0,), ix, False)[0]
    stop = threading.Event()

    def releaser():
        while not stop.is_set():
            release_resident(var)

    t = threading.Thread(target=releaser)
    t.start()
    try:
        with concurrent.futures.ThreadPoolExecutor(max_workers=6) as ex:
            got = list(ex.map(lambda _: _query(var, "mean", (0,), ix, True)[0], range(36)))
    finally:
        stop.set()
        t.join()
    for k, g in enumerate(got):
        _same(g, want, f"racing query {k}")
    release_resident(var)
    assert getattr(var, "_pyas_resident", None) is None


def _q(act, method, axis):
    """Set up a query as the reference's users do (active.method, axis)."""
    act.method = method
    act._axis = axis
    return act


def test_resident_plan_replay(gpu, monkeypatch):
    """Repeat box queries replay the cached device plan (_CachedQuery): the
    same results as a fresh query for every method, components mode and
    axis set, a new plan when the missing-data attributes change, and no
    plans left after release_resident."""
    from pyactivestorage_amd import active as A
    var = D.make_variable()
    nd = len(var.shape)
    built = []
    real = A._CachedQuery.__init__

    def spy(self, *a, **k):
        built.append(1)
        real(self, *a, **k)
    monkeypatch.setattr(A._CachedQuery, "__init__", spy)
    index = (slice(1, None),) + (slice(None),) * (nd - 1)
    try:
        for axis in (None, (0,), (nd - 1,), (0, nd - 1)):
            for method in ("mean", "sum", "min", "max"):
                want = _q(Active(var), method, axis)[index]
                act = _q(Active(var, resident=True), method, axis)
                first = act[index]
                n_built = len(built)
                for _ in range(2):
                    again = _q(act, method, axis)[index]
                    _same(again, want, f"{method} {axis} replay", "exact")
                _same(first, want, f"{method} {axis}", "exact")
                assert len(built) == n_built            # replays built nothing
                act.components = True
                comp = _q(act, method, axis)[index]
                ref_act = Active(var)
                ref_act.components = True
                ref = _q(ref_act, method, axis)[index]
                assert comp.keys() == ref.keys()
                for k in ref:
                    _same(comp[k], ref[k], f"{method} {axis} components {k}", "exact")
        store = var._pyas_resident
        n_plans = len(store["plans"])
        assert n_plans == 4                              # one per axis set (method-independent)
        var.attrs = dict(var.attrs, valid_max=np.array([50.0], dtype=var.dtype))
        want, _ = _query(var, "mean", None, index, False)
        got, _ = _query(var, "mean", None, index, True)
        _same(got, want, "changed valid_max", "exact")
        assert len(store["plans"]) == n_plans + 1
    finally:
        release_resident(var)
    assert getattr(var, "_pyas_resident", None) is None


def test_attach_resident_matches_file(gpu):
    """attach_resident: chunks a GPU producer already holds in
    HBM, in the resident slot layout, answer whole and partial-axis queries
    exactly as the variable's own bytes do; a misaligned pointer and a query
    on another device than the attached one raise instead of silently
    replacing the caller's store."""
    from pyactivestorage_amd.active import attach_resident
    from pyactivestorage_amd.device import DeviceBuffer
    var = D.make_variable()
    ref = D.make_variable()
    nd = len(var.shape)
    grid = [-(-s // c) for s, c in zip(var.shape, var.chunks)]
    nbytes = int(np.prod(var.chunks)) * np.dtype(var.dtype).itemsize
    stride = -(-nbytes // 256) * 256
    host = np.zeros(int(np.prod(grid)) * stride, dtype=np.uint8)
    for k, cc in enumerate(np.ndindex(*grid)):
        off, size = var.chunk_info(cc)
        host[k * stride: k * stride + size] = np.frombuffer(var.read(off, size), dtype=np.uint8)
    # the producer's buffer (the library's own allocation: this process's HIP
    # runtime is libpyas_hip's, no torch here)
    data = DeviceBuffer(gpu, host.nbytes)
    st = gpu.thread_stream()
    gpu.h2d(data.ptr, host, st)
    gpu.synchronize(st)
    with pytest.raises(ValueError, match="aligned"):
        attach_resident(var, data.ptr + 4, device=0, owner=data)
    attach_resident(var, data.ptr, device=0, owner=data)
    try:
        with pytest.raises(ValueError, match="already has a resident copy"):
            attach_resident(var, data.ptr, device=0, owner=data)
        half = tuple(slice(0, max(1, n // 2)) for n in var.shape)
        for method, axis, index in [("mean", None, (slice(None),) * nd), ("min", (0,), half),
                                    ("max", (nd - 1,), half), ("mean", (0, nd - 1), (slice(None),) * nd)]:
            want, _ = _query(ref, method, axis, index, False)
            got, read = _query(var, method, axis, index, True)
            assert read == 0, (method, axis)          # nothing from the variable's reader
            _same(got, want, f"attached {method} {axis}", "exact")
        from pyactivestorage_amd.active import _check_attached
        with pytest.raises(ValueError, match="attached on device 0"):
            _check_attached(var, 1)               # what a device-1 query meets first
    finally:
        release_resident(var)
    assert getattr(var, "_pyas_resident", None) is None
