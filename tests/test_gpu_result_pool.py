"""Pinned result arrays (device.Context.result_array): Active's formatted
values and mask are copied D2H into pinned blocks leased from a per-context
pool; a block returns to the pool when its array and every view of it are
gone, and beyond the pool's cap callers get pageable arrays."""
import gc

import numpy as np
import pytest

from pyactivestorage_amd.device import DeviceBuffer, _ResultPool

pytestmark = pytest.mark.gpu


def test_lease_returns_block(gpu):
    pool = _ResultPool(gpu, 8 << 20)
    a = pool.array(100_000, np.float32)          # 400 KB -> a 512 KiB block
    assert a.nbytes == 400_000 and pool.pinned == 512 << 10
    ptr = a.ctypes.data
    v = a.reshape(100, 1000)[::2]                 # a view keeps the lease
    del a
    gc.collect()
    assert not pool.free.get(512 << 10)
    del v
    gc.collect()
    assert pool.free[512 << 10] == [ptr]
    b = pool.array(70_000, np.float64)            # 560 KB: a 1 MiB block
    c = pool.array(120_000, np.float32)           # 480 KB: reuses the 512 KiB block
    assert c.ctypes.data == ptr and pool.pinned == (512 << 10) + (1 << 20)
    del b, c


def test_cap_and_small_arrays_are_pageable(gpu):
    pool = _ResultPool(gpu, 1 << 20)
    small = pool.array(100, np.float32)
    assert pool.pinned == 0 and small.flags.owndata
    keep = pool.array(200_000, np.float32)        # 800 KB: the whole cap
    over = pool.array(200_000, np.float32)        # over the cap: pageable
    assert pool.pinned == 1 << 20 and over.flags.owndata and not keep.flags.owndata


def test_d2h_into_pinned_result(gpu):
    n = 1 << 20
    src = np.arange(n, dtype=np.float32)
    buf = DeviceBuffer(gpu, src.nbytes)
    st = gpu.thread_stream()
    gpu.h2d(buf.ptr, src, st)
    out = gpu.result_array(n, np.float32)
    gpu.d2h(out, buf.ptr, st)
    gpu.synchronize(st)
    np.testing.assert_array_equal(out, src)
    buf.free()
