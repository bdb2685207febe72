"""pyas_format_partials (the device form of ``Active._format``, i.e. the
end of ``Active._from_storage``, ``activestorage/active.py:591-630``)
against the host formatting of the same partials through ``np.ma``.

Bit-exact: values (including NaN payload-free NaNs, ±inf, -0.0 and what
``np.ma``'s ``out / n`` leaves under the mask), mask, dtype and fill value,
for every dtype class and method, with counts of 0 (masked), NaN and
infinite sums, huge f64 sums (the safe-divide domain) and wrapping ints.
"""
import numpy as np
import pytest

from pyactivestorage_amd import engine
from pyactivestorage_amd.device import DeviceBuffer
from pyactivestorage_amd.dtypes import native, sum_dtype

pytestmark = pytest.mark.gpu

DTYPES = ["<f4", ">f4", "<f8", ">f8", "<i1", "<u1", "<i2", ">i2", "<u2", "<i4", "<u4", "<i8", "<u8"]


def _host(final, dt, method, components):
    """Active._format (pyactivestorage_amd/active.py), active.py:591-630."""
    cnt = np.ascontiguousarray(final["count"]).astype(np.int64)
    if method in ("sum", "mean"):
        vals = final["sum"].astype(native(dt) if dt.kind == "f" else sum_dtype(dt))
    else:
        vals = final[method].astype(native(dt))
    out = np.ma.MaskedArray(np.ascontiguousarray(vals), mask=(cnt == 0))
    n = np.ma.MaskedArray(cnt, mask=np.zeros(cnt.shape, dtype=bool))
    if components:
        return out, n
    with np.errstate(all="ignore"):
        return (out / n if method == "mean" else out), None


def _partials(dt, n, rng):
    f = np.zeros(n, engine.partial_dtype(dt))
    f["count"] = rng.integers(0, 6, n)
    if dt.kind == "f":
        big = 300 if dt.itemsize == 8 else 38
        s = rng.normal(size=n) * 10.0 ** rng.integers(-40, big, n)
        s[::17] = np.nan
        s[::19] = np.inf
        s[::23] = -np.inf
        s[::29] = -0.0
        if dt.itemsize == 8:
            s[::31] = 1.7e308          # |out| * tiny >= n for small n
        f["sum"] = s
        with np.errstate(all="ignore"):
            f["min"] = s.astype(dt).astype(np.float64)
            f["max"] = -s.astype(dt).astype(np.float64)
    else:
        info = np.iinfo(dt)
        if dt.kind == "i":
            s = rng.integers(-2 ** 62, 2 ** 62, n)
            s[::13] = np.iinfo(np.int64).min
        else:
            s = rng.integers(0, 2 ** 63, n).astype(np.uint64) * np.uint64(2)
        f["sum"] = s
        nat = native(dt)
        f["min"] = rng.integers(info.min, info.max, n, endpoint=True, dtype=nat).astype(f["min"].dtype)
        f["max"] = rng.integers(info.min, info.max, n, endpoint=True, dtype=nat).astype(f["max"].dtype)
    return f


def _same(a, b):
    assert a.dtype == b.dtype
    assert np.array_equal(np.ma.getmaskarray(a), np.ma.getmaskarray(b))
    assert a.data.tobytes() == b.data.tobytes()


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("method", ["sum", "min", "max", "mean"])
def test_format_matches_np_ma(gpu, dt, method):
    ctx = gpu
    dt = np.dtype(dt)
    rng = np.random.default_rng(abs(hash((dt.str, method))) % 2 ** 32)
    n = 4099
    final = _partials(dt, n, rng)
    st = ctx.thread_stream()
    src = DeviceBuffer(ctx, final.nbytes)
    ctx.h2d(src.ptr, final, st)
    vdt = engine.format_dtype(dt, method)
    vbuf, mbuf, cbuf = DeviceBuffer(ctx, n * vdt.itemsize), DeviceBuffer(ctx, n), DeviceBuffer(ctx, 8 * n)
    engine.format_partials(ctx, dt, src.ptr, n, method, vbuf.ptr, mbuf.ptr, cbuf.ptr, st)
    vals, mask, cnt = np.empty(n, vdt), np.empty(n, np.bool_), np.empty(n, np.int64)
    ctx.d2h(vals, vbuf.ptr, st)
    ctx.d2h(mask, mbuf.ptr, st)
    ctx.d2h(cnt, cbuf.ptr, st)
    ctx.synchronize(st)
    got = np.ma.MaskedArray(vals, mask=mask)
    want, _ = _host(final, dt, method, components=False)
    _same(got, want)
    assert got.fill_value == want.fill_value or (np.isnan(got.fill_value) and np.isnan(want.fill_value))
    np.testing.assert_array_equal(cnt, final["count"])


def test_format_refuses_bad_method(gpu):
    ctx = gpu
    from pyactivestorage_amd import _lib
    rc = ctx.lib.pyas_format_partials(ctx.handle, _lib.F32, 8, 1, 9, 8, 8, None, None)
    assert rc == _lib.EINVAL


@pytest.mark.parametrize("components", [False, True])
@pytest.mark.parametrize("method", ["mean", "sum", "min", "max"])
def test_active_axis_device_format_matches_host(method, components):
    """Active over a box query with partial axes formats on the device;
    the same partials formatted on the host give the same result."""
    from pyactivestorage_amd.active import Active
    from pyactivestorage_amd.variable import ChunkedVariable
    import os
    import tempfile
    rng = np.random.default_rng(5)
    shape, chunks = (12, 10, 9), (4, 3, 5)
    data = rng.uniform(0, 100, size=shape).astype("<f4")
    data[rng.random(shape) < 0.3] = -999.0
    data[:4, :3, :] = -999.0            # every element of some outputs masked
    path = os.path.join(tempfile.mkdtemp(), "v.chunks")
    index, pos = {}, 0
    with open(path, "wb") as fh:
        for cc in np.ndindex(*[-(-s // c) for s, c in zip(shape, chunks)]):
            block = np.full(chunks, -999.0, "<f4")
            sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(cc, chunks, shape))
            block[tuple(slice(0, x.stop - x.start) for x in sl)] = data[sl]
            fh.write(block.tobytes())
            index[cc] = (pos, block.nbytes)
            pos += block.nbytes
    var = ChunkedVariable(name="v", shape=shape, chunks=chunks, dtype=np.dtype("<f4"), chunk_index=index,
                          attrs={"_FillValue": np.array([-999.0], "<f4")}, filename=path)
    for axis in [(0,), (1,), (2,), (0, 1), (1, 2), (0, 2)]:
        a = Active(var, axis=axis)
        a.components = components
        a.method = method
        got = a[1:11, :, 2:9]
        b = Active(var, axis=axis)
        b.components = components
        b.method = method
        b._format_device = lambda ctx, st, fin, n, shape, _b=b: _b._format(_host_final(ctx, st, fin, n, _b).reshape(shape), shape)
        want = b[1:11, :, 2:9]
        if components:
            key = "sum" if method == "mean" else method
            _same(got[key], want[key])
            _same(got["n"], want["n"])
        else:
            _same(got, want)


def _host_final(ctx, st, fin, n, act):
    final = np.zeros(n, dtype=engine.partial_dtype(act.ds.dtype))
    ctx.d2h(final, fin.ptr, st)
    ctx.synchronize(st)
    return final
