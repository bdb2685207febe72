"""NumPy's sign of a zero min/max on the device (pyas_zero_sign_chunks /
pyas_zero_sign_seq, rule from zerosign.py).

Per chunk (``storage.py:99-100``): the drop-in's per-call path and the
coalesced pool path return the reference's +0.0 / -0.0 (the golden cases of
``tests/golden`` hold 420 such chunks made by the reference itself).  Across
chunks (``active.py:575-598``): ``Active`` reduces the per-chunk results in
the ``out`` array's C order with ``np.ma.min/max``, so the final zero's sign
follows the same rule over the chunk sequence; here it is checked against a
NumPy restatement of that combine.
"""
import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import storage as pas
from pyactivestorage_amd.active import Active
from pyactivestorage_amd.variable import ChunkedVariable
from pyactivestorage_amd.zerosign import tie_rule

pytestmark = pytest.mark.gpu


def _chunk(rng, shape, dt, pattern, n_zero=25):
    n = int(np.prod(shape))
    if pattern == "zeros":
        a = np.zeros(n, dtype=dt)
    else:
        a = rng.uniform(0.5, 9.0, n).astype(dt) * (1 if pattern == "min0" else -1)
    a[rng.choice(n, n_zero, replace=False)] = np.where(rng.random(n_zero) < 0.5, -0.0, 0.0)
    a[rng.choice(n, 10, replace=False)] = -999.0
    return a.reshape(shape)


@pytest.mark.parametrize("dt", ["<f4", ">f8"])
@pytest.mark.parametrize("pattern", ["min0", "max0", "zeros"])
def test_per_call_chunk_sign(gpu, dt, pattern):
    rng = np.random.default_rng(len(dt) * 7 + len(pattern))
    shape = (12, 20, 70)                               # > one 8192-element iterator piece
    full = (slice(None),) * 3
    box = (slice(1, 11), slice(2, 19), slice(0, 66, 3))
    for trial in range(6):
        a = _chunk(rng, shape, np.dtype(dt), pattern)
        raw = a.tobytes()
        for miss in ((None, None, None, None), (np.dtype(dt).type(-999.0), None, None, None)):
            for sel in ((full,) if miss[0] is None else (full, box)):
                for method in (np.ma.min, np.ma.max, np.min, np.max):
                    want, _ = ref.reduce_chunk_bytes(raw, None, None, miss, dt, shape, "C", sel, (0, 1, 2), method)
                    got, _ = pas.reduce_chunk_bytes(raw, None, None, miss, dt, shape, "C", sel, (0, 1, 2), method)
                    w, g = np.ma.getdata(want).reshape(-1)[0], np.ma.getdata(got).reshape(-1)[0]
                    assert w == g or (np.isnan(w) and np.isnan(g)), (trial, method, w, g)
                    if w == 0:
                        assert np.signbit(w) == np.signbit(g), (trial, miss, sel, method.__name__, w, g)


def _reference_combine(arr, chunks, miss_fill, method):
    """active.py:575-598 over storage.py's per-chunk results: per-chunk
    np.ma.min/max into `out` (the variable dtype, masked where a chunk is
    all masked), then np.ma.min/max over `out`."""
    grid = tuple(s // c for s, c in zip(arr.shape, chunks))
    out = np.ma.masked_all(grid, dtype=arr.dtype)
    for cc in np.ndindex(*grid):
        sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(cc, chunks))
        tmp = np.ma.masked_equal(arr[sl], miss_fill)
        r = method(tmp, axis=(0, 1, 2), keepdims=True)
        out[cc] = r.reshape(())
    return method(out, axis=(0, 1, 2), keepdims=True)


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("kind", ["min", "max"])
@pytest.mark.parametrize("resident", [False, True])
def test_active_combine_sign(gpu, dt, kind, resident):
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(3 + len(kind) + resident)
    shape, chunks = (8, 12, 40), (4, 4, 10)
    method = np.ma.min if kind == "min" else np.ma.max
    for trial in range(5):
        a = np.full(shape, 5.0 if kind == "min" else -5.0, dtype=dt)
        n = a.size
        z = rng.choice(n, 30, replace=False)
        a.reshape(-1)[z] = np.where(rng.random(30) < 0.5, -0.0, 0.0)
        a.reshape(-1)[rng.choice(n, 10, replace=False)] = -999.0
        blobs, index, pos = [], {}, 0
        grid = [s // c for s, c in zip(shape, chunks)]
        for cc in np.ndindex(*grid):
            sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(cc, chunks))
            b = np.ascontiguousarray(a[sl]).tobytes()
            index[cc] = (pos, len(b))
            blobs.append(b)
            pos += len(b)
        data = b"".join(blobs)
        var = ChunkedVariable(name="v", shape=shape, chunks=chunks, dtype=dt, chunk_index=index,
                              attrs={"_FillValue": np.array([-999.0], dtype=dt)},
                              reader=lambda off, size: data[off:off + size])
        act = Active(var, resident=resident)
        act.method = kind
        got = act[...]
        want = _reference_combine(a, chunks, np.dtype(dt).type(-999.0), method)
        w, g = np.ma.getdata(want).reshape(-1)[0], np.ma.getdata(got).reshape(-1)[0]
        assert w == g == 0, (trial, w, g)
        assert np.signbit(w) == np.signbit(g), (trial, kind, w, g)
