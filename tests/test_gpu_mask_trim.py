"""Mask-rule trimming (pyas_capi.hip ``trim_mask``): an equality rule
(_FillValue / missing_value) whose interval lies wholly beyond a valid_min /
valid_max threshold is dropped before launch, so the kernels run a mode with
fewer compares (``mask_mode``).  The set of masked values must not change:
``storage.py:126-153`` masks the union of all four rules.  Boundary cases put
the fill value exactly on, just inside and just outside each threshold, for
float and integer dtypes, whole-chunk and partial-axis reductions, plain and
shuffled chunks (every kernel family that picks a mask mode).
"""
import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import storage as pas
from tests._compare import assert_counts, assert_same, shuffle_bytes

pytestmark = pytest.mark.gpu

SHAPE = (8, 16, 32)


def _cases():
    out = []
    for dt in ("<f4", "<f8", "<i4", "<u4", ">f4"):
        lo, hi = 10, 90
        for fill in (lo - 1, lo, lo + 1, hi - 1, hi, hi + 1, 50):
            out.append((dt, (fill, None, lo, None)))     # valid_min only
            out.append((dt, (fill, None, None, hi)))     # valid_max only
            out.append((dt, (fill, None, lo, hi)))       # valid range
            out.append((dt, (None, fill, lo, hi)))       # missing_value (second rule)
            out.append((dt, (fill, fill + 1, lo, hi)))   # both equality rules
    return out


CASES = _cases()


@pytest.mark.parametrize("case", range(len(CASES)))
def test_trimmed_mask_matches_oracle(gpu, case):
    dt, miss = CASES[case]
    np_dt = np.dtype(dt)
    rng = np.random.default_rng(case)
    arr = rng.integers(0, 100, size=SHAPE).astype(np_dt)
    arr.reshape(-1)[::7] = miss[0] if miss[0] is not None else miss[1]
    if np_dt.kind == "f":
        arr.reshape(-1)[3] = np.nan
    miss = tuple(None if m is None else np_dt.type(m) for m in miss)
    sel = tuple(slice(0, n, 1) for n in SHAPE)
    es = np_dt.itemsize
    for shuf in (False, True):
        raw = shuffle_bytes(arr, es) if shuf else arr.tobytes()
        rf = [ref.Shuffle(es)] if shuf else None
        gf = [pas.Shuffle(es)] if shuf else None
        for axis in ((0, 1, 2), (0,), (2,), (0, 1)):
            for method in (np.ma.sum, np.ma.min, np.ma.max):
                what = f"{dt} miss={miss} shuf={shuf} axis={axis} {method.__name__}"
                want, wn = ref.reduce_chunk_bytes(raw, None, rf, miss, dt, SHAPE, "C", sel, axis, method)
                got, gn = pas.reduce_chunk_bytes(raw, None, gf, miss, dt, SHAPE, "C", sel, axis, method)
                vals, _ = ref.reduce_chunk_bytes(raw, None, rf, miss, dt, SHAPE, "C", sel, axis, None)
                with np.errstate(all="ignore"):
                    abs_sum = np.ma.sum(np.abs(np.ma.asarray(vals).astype(np.float64)), axis=axis,
                                        keepdims=True)
                assert_same(want, got, method.__name__, np.ma.filled(abs_sum, 0), what)
                assert_counts(wn, gn, what)
