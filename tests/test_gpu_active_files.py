"""``Active(path, ncvar)`` straight on the reference's test files
(tests/golden/nc, copies of the reference's tests/test_data): the HDF5
reader supplies the metadata, the native pread ring the chunk bytes, the
GPU the rest.  Expected values are the literals hard-coded in the
reference's tests (file:line per case); the axis sweep must equal the
ChunkedVariable path (tests/test_gpu_active.py), which is pinned to the
oracle.
"""
import itertools
import os

import numpy as np
import pytest

from pyactivestorage_amd.active import Active
from tests.test_gpu_active import variable

pytestmark = pytest.mark.gpu

NC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nc")


def P(name):
    return os.path.join(NC, name)


@pytest.mark.parametrize("inflate", ["device", "host"])
def test_known_answers_from_files(gpu, inflate, monkeypatch):
    """zlib chunks inflated by pyas_inflate and by the host reader threads
    (pyas_read_ranges_zlib) give the reference's literals alike."""
    monkeypatch.setenv("PYAS_ACTIVE_INFLATE", inflate)
    a = Active(P("cesm2_native.nc"), "TREFHT")             # test_bigger_data.py:261-284
    a.method = "mean"
    a.components = True
    r = a[4:5, 1:2]
    np.testing.assert_allclose(r["sum"], np.array([[[2368.3232]]], dtype="float32"), rtol=1e-6)
    np.testing.assert_array_equal(r["n"], np.array([[[8]]]))
    a = Active(P("daily_data.nc"), "ta")                   # test_bigger_data.py:287-310
    a.method = "mean"
    a.components = True
    r = a[4:5, 1:2]
    np.testing.assert_array_equal(r["sum"], np.array([[[[1515.9822]]]], dtype="float32"))
    a = Active(P("daily_data_masked.nc"), "ta")            # test_bigger_data.py:373-389
    assert a.min()[:] == 245.0020751953125
    a = Active(P("test1.nc"), "tas")                       # test_active_axis.py:94-116
    assert a.min(axis=(0, 2))[...][0][0][0] == 209.44680786132812
    assert Active(P("test1.nc"), "tas").max(axis=(0, 2))[...][0][0][0] == 255.54661560058594
    assert Active(P("CMIP6-test.nc"), "tas").min(axis=(0, 1))[...][0][0][0] == 206.40918
    a = Active(P("obs4MIPS_CERES-EBAF_L3B_Ed2-8_rlut.nc"), "rlut")   # test_compression.py:149
    a._method = "min"
    assert a[0:2, 4:6, 7:9] == 124.0


@pytest.mark.parametrize("inflate", [True, False, "auto"])
@pytest.mark.parametrize("key", ["test1.nc:tas", "cesm2_native.nc:TREFHT", "CMIP6-test.nc:tas"])
def test_file_path_equals_variable_path(gpu, key, inflate):
    f, name = key.split(":")
    v = variable(key)
    nd = len(v.shape)
    for axis in [None] + [c for k in range(1, nd) for c in itertools.combinations(range(nd), k)]:
        for method in ("mean", "min", "max"):
            index = tuple(slice(n // 4, n) for n in v.shape)
            want = getattr(Active(v), method)(axis=axis)[index]
            got = getattr(Active(P(f), name, device_inflate=inflate), method)(axis=axis)[index]
            np.testing.assert_array_equal(np.ma.getmaskarray(got), np.ma.getmaskarray(want))
            np.testing.assert_array_equal(np.ma.getdata(got), np.ma.getdata(want))
