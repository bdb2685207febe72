"""GPU parity of the LDS row layout of ``k_axes_dense`` (modes 4/5/6: the
innermost dim reduced, one run of <= 256 B per output, staged through LDS
with 1, 2 or 4 lanes per output) against the oracle, with the lane count
forced through ``PYAS_ROW_LDS`` (read per call by the host planner).

Reference semantics: ``storage.py:95-100`` (``chunk[sel]``, mask,
``method(axis, keepdims=True)``, ``np.ma.count``); the axis sweep follows
``tests/unit/test_active_axis.py:30-78``.  Shapes cover runs of 1-16
vectors, odd vector counts (the planner drops to fewer lanes), output
counts that leave a partial last tile, and big-endian data.
"""
import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import storage as pas
from tests._compare import assert_counts, assert_same
from tests.test_gpu_axes_dense import _data

pytestmark = pytest.mark.gpu

# (shape, axis): the reduced dims are the trailing ones, so RO == 1
CASES = [((3, 5, 12), (2,)), ((5, 7, 20), (2,)), ((2, 4, 64), (2,)), ((9, 33, 16), (2,)),
         ((4, 3, 8, 8), (2, 3)), ((70, 4), (1,)), ((3, 5, 6), (2,))]
DTYPES = ["<f4", ">f4", "<f8", "<i2", ">i4", "u1", "<u8"]
METHODS = [np.ma.sum, np.ma.min, np.ma.max, np.ma.mean]


@pytest.mark.parametrize("lanes", ["0", "1", "2", "4"])
@pytest.mark.parametrize("dt", DTYPES)
def test_row_lds_matches_oracle(gpu, monkeypatch, lanes, dt):
    monkeypatch.setenv("PYAS_ROW_LDS", lanes)
    for ci, (shape, axis) in enumerate(CASES):
        rng = np.random.default_rng(ci)
        arr = _data(dt, shape, rng, nan=(ci % 2 == 0))
        raw = arr.tobytes()
        sel = tuple(slice(0, n, 1) for n in shape)
        for miss in [(None, None, None, None), (42, None, 0, 90)]:
            masked_sel, _ = ref.reduce_chunk_bytes(raw, None, None, miss, dt, shape, "C", sel, axis, None)
            with np.errstate(all="ignore"):
                abs_sum = np.ma.sum(np.abs(np.ma.asarray(masked_sel).astype(np.float64)),
                                    axis=axis, keepdims=True)
            for method in METHODS:
                what = f"lanes={lanes} {dt} {shape} miss={miss} axis={axis} {method.__name__}"
                want, wn = ref.reduce_chunk_bytes(raw, None, None, miss, dt, shape, "C", sel, axis, method)
                got, gn = pas.reduce_chunk_bytes(raw, None, None, miss, dt, shape, "C", sel, axis, method)
                assert_same(want, got, method.__name__, np.ma.filled(abs_sum, 0), what)
                assert_counts(wn, gn, what)
