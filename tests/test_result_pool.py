"""Host logic of the pinned result pool (device._ResultPool) with a stand-in
allocator: leases return blocks when the last view of a result array is
gone, blocks are reused by size class, the cap and the small-array cutoff
fall back to pageable arrays.  The GPU form is tests/test_gpu_result_pool.py."""
import ctypes
import gc
import threading

import numpy as np

from pyactivestorage_amd.device import _ResultPool


class _FakeLib:
    def __init__(self):
        self.blocks = []

    def pyas_host_alloc(self, handle, size, out):
        buf = ctypes.create_string_buffer(size)
        self.blocks.append(buf)
        ctypes.cast(out, ctypes.POINTER(ctypes.c_void_p))[0] = ctypes.addressof(buf)
        return 0


class _FakeCtx:
    def __init__(self):
        self.lib = _FakeLib()
        self.handle = None


def test_lease_and_reuse():
    ctx = _FakeCtx()
    pool = _ResultPool(ctx, 4 << 20)
    a = pool.array(70_000, np.float64)            # 560 KB -> 1 MiB block
    a[:] = np.arange(a.size)
    assert pool.pinned == 1 << 20 and not a.flags.owndata
    m = np.ma.MaskedArray(a.reshape(700, 100), mask=np.zeros((700, 100), bool))
    ptr = a.ctypes.data
    del a
    gc.collect()
    assert not pool.free.get(1 << 20)             # the masked array still holds it
    assert float(m[699, 99]) == 69_999.0
    del m
    gc.collect()
    assert pool.free[1 << 20] == [ptr]
    b = pool.array(100_000, np.float64)           # 800 KB: the same size class
    assert b.ctypes.data == ptr and len(ctx.lib.blocks) == 1


def test_cap_and_cutoff():
    pool = _ResultPool(_FakeCtx(), 1 << 20)
    assert pool.array(10, np.int64).flags.owndata           # under MIN_BYTES
    keep = pool.array(200_000, np.float32)                  # 1 MiB block: the cap
    over = pool.array(200_000, np.float32)
    assert not keep.flags.owndata and over.flags.owndata and pool.pinned == 1 << 20
    off = _ResultPool(_FakeCtx(), 0)
    assert off.array(1 << 20, np.uint8).flags.owndata


def test_threads_share_the_pool():
    ctx = _FakeCtx()
    pool = _ResultPool(ctx, 64 << 20)
    errs = []

    def work(k):
        try:
            for i in range(50):
                x = pool.array(100_000 + k, np.float32)
                x[:] = k
                assert (x == k).all()
                del x
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
    ts = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    gc.collect()
    assert not errs
    assert pool.pinned <= 8 * (512 << 10)         # at most one block per thread at a time
