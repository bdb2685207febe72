"""The zero-sign tie rule derived from this host's NumPy (zerosign.py),
checked against NumPy itself on the CPU.

``storage.py:99-100`` returns ``np.ma.min/max(..., keepdims=True)``; when the
extreme is zero and both signed zeros occur, NumPy's result depends on its
reduction loop.  :func:`zerosign.emulate` restates the contiguous loop;
:func:`zerosign.predict` is the key algorithm the device runs
(``pyas_tie_chunks`` / ``pyas_tie_grid``).  Both must give NumPy's sign:
for contiguous data (every masked chunk: ``np.ma`` reduces ``filled()``, a
copy), for any axis subset, for F-ordered and big-endian arrays, for strided
and reversed views (an unmasked ``chunk[sel]`` is reduced as the view), for
index-list results, and for reduce calls longer than one iterator buffer
(``np.getbufsize()``).
"""
import itertools

import numpy as np
import pytest

from pyactivestorage_amd import zerosign


def _plant(rng, shape, dt, op, k):
    a = (rng.uniform(0.5, 2.0, shape) * (1 if op is np.min else -1)).astype(dt)
    flat = a.reshape(-1)
    pos = rng.integers(0, flat.size, k)
    flat[pos] = np.where(rng.random(k) < 0.5, -0.0, 0.0)
    return a


@pytest.mark.parametrize("dt", ["f4", "f8"])
def test_rule_derived_and_sane(dt):
    r = zerosign.tie_rule(dt)
    assert r is not None
    assert sorted(r.order) == list(range(r.lanes)) and r.piece == np.getbufsize()
    assert [r.rank[lane] for lane in r.order] == list(range(r.lanes))
    assert zerosign.tie_rule("i4") is None


@pytest.mark.parametrize("dt", ["f4", "f8"])
@pytest.mark.parametrize("op", [np.min, np.max])
def test_rule_matches_numpy_flat_and_3d(dt, op):
    r = zerosign.tie_rule(dt)
    rng = np.random.default_rng(11 if op is np.min else 12)
    n_checked = 0
    for trial in range(150):
        if trial % 3 == 0:
            shape = tuple(int(x) for x in rng.integers(2, 48, 3))
        else:
            shape = (int(rng.integers(1, 3 * r.piece)),)
        a = _plant(rng, shape, np.dtype(dt), op, int(rng.integers(1, 9)))
        got = zerosign.emulate(a, op, r.lanes, r.order, r.piece)
        want = op(a, axis=tuple(range(a.ndim)), keepdims=True)
        if got is None:
            assert want.reshape(-1)[0] != 0
            continue
        n_checked += 1
        assert got == bool(np.signbit(want).reshape(-1)[0]), (trial, shape)
    assert n_checked > 100


@pytest.mark.parametrize("dt", ["f4", "f8"])
def test_rule_matches_masked_reduction(dt):
    """np.ma.min/max of a masked array (what storage.py reduces when any
    missing-data attribute is set): masked elements become +/-inf and never
    tie with zero."""
    r = zerosign.tie_rule(dt)
    rng = np.random.default_rng(5)
    for op, mop in ((np.min, np.ma.min), (np.max, np.ma.max)):
        for trial in range(60):
            shape = tuple(int(x) for x in rng.integers(2, 40, 3))
            a = _plant(rng, shape, np.dtype(dt), op, int(rng.integers(2, 9)))
            fill = np.dtype(dt).type(-999.0)
            a.reshape(-1)[rng.integers(0, a.size, 5)] = fill
            m = np.ma.masked_equal(a, fill)
            want = mop(m, axis=(0, 1, 2), keepdims=True)
            filled = m.filled(np.inf if op is np.min else -np.inf)
            got = zerosign.emulate(filled, op, r.lanes, r.order, r.piece)
            if got is not None:
                assert got == bool(np.signbit(np.ma.getdata(want)).reshape(-1)[0]), trial


def _axis_sets(nd):
    out = [None]
    for k in range(1, nd + 1):
        out += list(itertools.combinations(range(nd), k))
    return out


def _dense(rng, shape, dt, op):
    a = (rng.uniform(0.5, 2.0, shape) * (1 if op is np.min else -1)).astype(dt)
    f = a.reshape(-1)
    z = rng.random(f.size) < rng.choice([0.002, 0.02, 0.2, 0.6])
    f[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
    return a


def _check_predict(a, axis, op):
    """The key algorithm (full keys) and the device's early-stopping
    backward scan (k_tie_scan, step 1 and a wave-sized step) against NumPy."""
    got = op(a, axis=axis, keepdims=True)
    rule = zerosign.tie_rule(a.dtype)
    pred = zerosign.predict(a, axis, op, rule)
    scans = [zerosign.predict_scan(a, axis, op, rule, step)[0] for step in (1, 64)]
    n = 0
    for o, p in pred.items():
        if got[o] == 0:
            n += 1
            assert p is not None and p == bool(np.signbit(got[o])), (a.shape, a.strides, axis, o)
        else:
            assert p is None
        assert all(sc[o] == p for sc in scans), (a.shape, a.strides, axis, o, p, [sc[o] for sc in scans])
    return n


@pytest.mark.parametrize("kind", ["C", "F", "BE"])
def test_keys_match_numpy_contiguous(kind):
    rng = np.random.default_rng({"C": 1, "F": 2, "BE": 3}[kind])
    n = 0
    for _ in range(60):
        op = np.min if rng.random() < .5 else np.max
        dt = str(rng.choice(["f4", "f8"]))
        nd = int(rng.integers(1, 5))
        shape = tuple(int(rng.choice([1, 2, 3, 5, 7, 16, 17, 33, 64])) for _ in range(nd))
        while np.prod(shape) > 20000:
            shape = shape[1:]
        a = _dense(rng, shape, dt, op)
        if kind == "F":
            a = np.asfortranarray(a)
        if kind == "BE":
            a = a.astype(a.dtype.newbyteorder(">"))
        axes = _axis_sets(a.ndim)
        n += _check_predict(a, axes[int(rng.integers(len(axes)))], op)
    assert n > 300


@pytest.mark.parametrize("kind", ["view", "view-BE", "list"])
def test_keys_match_numpy_views(kind):
    """Strided and reversed views (the acc loop when the inner reduced dim
    is not contiguous), non-native views (buffered) and index-list copies
    (laid out with the listed dim outermost)."""
    rng = np.random.default_rng({"view": 4, "view-BE": 5, "list": 6}[kind])
    n = 0
    for _ in range(80):
        op = np.min if rng.random() < .5 else np.max
        dt = str(rng.choice(["f4", "f8"]))
        nd = int(rng.integers(1, 4))
        shape = tuple(int(rng.choice([4, 8, 16, 33, 64, 300])) for _ in range(nd))
        while np.prod(shape) > 40000:
            shape = shape[1:]
        base = _dense(rng, shape, dt, op)
        if kind == "view-BE":
            base = base.astype(base.dtype.newbyteorder(">"))
        sl = []
        for s in shape:
            st = int(rng.choice([1, 1, 2, 3])) * (-1 if rng.random() < .3 else 1)
            a0 = int(rng.integers(0, s // 2))
            a1 = int(rng.integers(a0 + 1, s + 1))
            sl.append(slice(a0, a1, st) if st > 0 else slice(a1 - 1, a0 - 1 if a0 > 0 else None, st))
        a = base[tuple(sl)]
        if kind == "list":
            d = int(rng.integers(0, a.ndim))
            idx = np.sort(rng.choice(a.shape[d], size=max(1, a.shape[d] // 2), replace=False))
            a = a[tuple(idx if i == d else slice(None) for i in range(a.ndim))]
        axes = _axis_sets(a.ndim)
        n += _check_predict(a, axes[int(rng.integers(len(axes)))], op)
    assert n > 100


@pytest.mark.parametrize("dt", ["<f4", ">f8"])
def test_keys_match_numpy_long_calls(dt):
    """Reduce calls longer than np.getbufsize(): pieces inside each call."""
    rng = np.random.default_rng(9)
    for shape, axis, key in [((3, 2, 20000), (0, 2), None), ((2, 3, 9000), (1, 2), None),
                             ((40000,), None, (slice(None, None, 2),)),
                             ((4, 30000), (1,), (slice(None), slice(None, None, 3))),
                             ((4, 3, 5000), (1, 2), (slice(None), slice(None), slice(0, 4500))),
                             ((3, 20000), (1,), (slice(None), slice(None, None, -1)))]:
        for op in (np.min, np.max):
            for dens in (0.0005, 0.3):
                a = (rng.uniform(0.5, 2, shape) * (1 if op is np.min else -1)).astype(dt)
                f = a.reshape(-1)
                z = rng.random(f.size) < dens
                f[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
                _check_predict(a[key] if key else a, axis, op)


def test_geometry_of_selections():
    """zerosign.geometry: the view flag only for unmasked slice selections,
    list dims outermost, F-ordered chunks as reversed dims, byte order."""
    from pyactivestorage_amd import selection
    shape = (4, 6, 8)
    cs = selection.normalize((slice(1, 3), slice(None, None, -2), slice(None)), shape)
    g = zerosign.geometry(shape, "C", cs, False, "<f4")
    assert list(g.perm[:3]) == [0, 1, 2] and g.flags == zerosign.GEOM_VIEW
    g = zerosign.geometry(shape, "C", cs, True, ">f4")
    assert g.flags == zerosign.GEOM_BUFFERED
    cs = selection.normalize((slice(None), [1, 3, 4], slice(None)), shape)
    g = zerosign.geometry(shape, "C", cs, False, "<f8")
    assert list(g.perm[:3]) == [1, 0, 2] and g.flags == 0
    g = zerosign.geometry(shape, "F", cs, False, "<f8")   # user dims (1, 2, 0) in memory order
    assert list(g.perm[:3]) == [1, 0, 2]
    assert zerosign.grid_lr((16, 16, 16), {0, 1, 2}) == 4096
    assert zerosign.grid_lr((16, 1024, 16), {0, 2}) == 16
    assert zerosign.grid_lr((16, 1024, 1024), {0}) == 1
    assert zerosign.grid_lr((16, 1, 16), {0, 2}) == 256


@pytest.mark.parametrize("dt", ["f4", "f8"])
def test_keys_match_numpy_copied_first_fill(dt):
    """An unmasked view whose reduced inner dim is strided runs NumPy's
    strided loop, except for the runs of the first buffer fill when that
    fill spans more than one kept iteration dim: NumPy copies those to a
    contiguous buffer (zerosign.call_structure's n_copy)."""
    rng = np.random.default_rng(21)
    S = slice(None)
    cases = [((12, 20, 70), (slice(1, 11), slice(2, 19), slice(0, 66, 3)), (2,)),
             ((12, 20, 70), (S, slice(2, 19), slice(0, 66, 3)), (2,)),
             ((4, 30, 600), (S, slice(0, 29), slice(0, 600, 3)), (2,)),
             ((3, 4, 5, 70), (S, S, slice(0, 4), slice(0, 66, 3)), (3,)),
             ((3, 140, 128), (S, slice(0, 129), slice(None, None, 2)), (2,)),
             ((3, 140, 128), (S, slice(0, 127), slice(None, None, 2)), (2,)),
             ((6, 20, 70), (S, slice(2, 19), slice(0, 66, 3)), (0, 2)),
             ((5, 9, 70), (S, slice(1, 8), slice(65, 2, -2)), (2,))]
    n = 0
    for shape, key, axis in cases:
        for _ in range(3):
            a = _dense(rng, shape, dt, np.min)
            n += _check_predict(a[key], axis, np.min)
    assert n > 500


def test_missing_tie_rule_is_reported_once(monkeypatch):
    """when no rule reproduces the host's NumPy, the
    context says so (RuntimeWarning once per dtype and process, and the
    per-dtype flag Context.tie_signs_exact is built from the same list)."""
    import warnings

    from pyactivestorage_amd import device, zerosign
    real = zerosign.tie_rule
    monkeypatch.setattr(zerosign, "tie_rule", lambda dt: None if np.dtype(dt).itemsize == 8 else real(dt))
    monkeypatch.setattr(device, "_TIE_WARNED", set())
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        first = device.host_tie_rules()
        again = device.host_tie_rules()
    msgs = [str(w.message) for w in rec if issubclass(w.category, RuntimeWarning)]
    assert len(msgs) == 1 and "f8" in msgs[0], msgs
    assert [(dt, r is None) for _, dt, r in first] == [("f4", real("f4") is None), ("f8", True)]
    assert [(dt, r is None) for _, dt, r in again] == [(dt, r is None) for _, dt, r in first]


def test_scan_stops_early_on_zero_heavy_data():
    """The backward scan reads only a few elements per output when zeros are
    dense (the cost the device pass pays on precipitation-like data)."""
    rng = np.random.default_rng(31)
    a = rng.uniform(1, 10, (16, 16, 256)).astype("f4")
    z = rng.random(a.shape) < 0.5
    a[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
    rule = zerosign.tie_rule("f4")
    for axis in (None, (0,), (2,), (1, 2)):
        res, scanned = zerosign.predict_scan(a, axis, np.min, rule)
        want = zerosign.predict(a, axis, np.min, rule)
        assert res == want
        n_red = a.size // len(res)
        assert np.mean(list(scanned.values())) < 0.2 * n_red, (axis, np.mean(list(scanned.values())), n_red)
