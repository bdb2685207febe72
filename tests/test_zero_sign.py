"""The zero-sign tie rule derived from this host's NumPy (zerosign.py),
checked against NumPy itself on the CPU.

``storage.py:99-100`` returns ``np.ma.min/max(..., keepdims=True)``; when the
extreme is zero and both signed zeros occur, NumPy's result depends on its
reduction loop.  :func:`zerosign.emulate` is the rule the device applies
(``pyas_zero_sign_chunks``); it must give NumPy's sign for contiguous data
(every masked chunk: ``np.ma`` reduces ``filled()``, a C-ordered copy), for
3-D arrays reduced over all axes, and for data longer than one iterator
buffer (``np.getbufsize()``).
"""
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
