"""pyas_reduce_sharded: several GPUs driven from one process through the C
ABI (active.py:557-598 across devices: per-device reduce, ONE RCCL
all-gather of the 32-byte totals, a device-order fold on every device).

On a one-GPU box the entry runs at ndev = 1 and must give the bytes of
pyas_reduce_chunks' total; with two or more visible GPUs the chunk list is
also split over devices and compared with the single-device combine
(count/min/max exact, sum within 1e-6).
"""
import ctypes

import numpy as np
import pytest

from pyactivestorage_amd import _lib, engine
from pyactivestorage_amd.batch import ReductionPlan
from pyactivestorage_amd.device import DeviceBuffer, get_context

pytestmark = pytest.mark.gpu

MISSING = (np.float32(-999.0), None, np.float32(1000.0), np.float32(5e8))


def _data(torch, dev, chunk_range=None):
    from pyactivestorage_amd.synthetic import chunk_major_device
    return chunk_major_device(torch, (256, 256, 256), (64, 64, 64), np.float32, dev, chunk_range=chunk_range,
                              fill=-999.0, fill_frac=0.01)


def _arr(ctype, vals):
    return (ctype * len(vals))(*vals)


def _sharded(ctxs, plans, streams, flags=1):
    n = len(ctxs)
    outs = [DeviceBuffer(c, (n + 1) * _lib.PARTIAL_NBYTES) for c in ctxs]
    lib = ctxs[0].lib
    rc = lib.pyas_reduce_sharded(
        _arr(ctypes.c_void_p, [c.handle for c in ctxs]),
        _arr(ctypes.c_void_p, [ctypes.addressof(p.batch) for p in plans]),
        _arr(ctypes.c_void_p, [ctypes.addressof(p.mask_up.struct) for p in plans]),
        n, flags, _arr(ctypes.c_void_p, [o.ptr for o in outs]), _arr(ctypes.c_void_p, streams))
    _lib.check(rc, "pyas_reduce_sharded")
    res = []
    for c, o, s in zip(ctxs, outs, streams):
        host = np.zeros(n + 1, dtype=engine.partial_dtype(np.float32))
        c.d2h(host, o.ptr, s)
        c.synchronize(s)
        res.append(host)
    return res


def test_one_device_equals_reduce_chunks(gpu):
    import torch
    dev = torch.device("cuda", 0)
    data, offsets, _ = _data(torch, dev)
    st = torch.cuda.current_stream().cuda_stream
    plan = ReductionPlan(gpu, np.float32, (64, 64, 64), data.data_ptr(), offsets, missing=MISSING, stream=st)
    plan.launch(st, chunk_partials=False)
    want = plan.read_total(st)
    for _ in range(3):   # the communicator is created once and reused
        got = _sharded([gpu], [plan], [st])[0]
        assert got[0].tobytes() == want.tobytes()
        assert got[1].tobytes() == want.tobytes()
    assert want["count"][0] > 0


def test_argument_errors(gpu):
    lib = gpu.lib
    assert lib.pyas_reduce_sharded(None, None, None, 0, 0, None, None) == _lib.EINVAL
    import torch
    dev = torch.device("cuda", 0)
    data, offsets, _ = _data(torch, dev, chunk_range=(0, 4))
    st = torch.cuda.current_stream().cuda_stream
    plan = ReductionPlan(gpu, np.float32, (64, 64, 64), data.data_ptr(), offsets, missing=MISSING, stream=st)
    out = DeviceBuffer(gpu, 3 * _lib.PARTIAL_NBYTES)
    rc = lib.pyas_reduce_sharded(_arr(ctypes.c_void_p, [gpu.handle, gpu.handle]),
                                 _arr(ctypes.c_void_p, [ctypes.addressof(plan.batch)] * 2), None, 2, 0,
                                 _arr(ctypes.c_void_p, [out.ptr, out.ptr]), _arr(ctypes.c_void_p, [st, st]))
    assert rc == _lib.EINVAL and b"appears twice" in lib.pyas_last_error()


def test_several_devices_equal_one(gpu):
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU visible: the ndev > 1 exchange runs on multi-GPU nodes only")
    n_chunks = 64
    from pyactivestorage_amd.distributed import equal_ranges
    ctxs, plans, streams, keep = [], [], [], []
    for k, (lo, hi) in enumerate(equal_ranges(n_chunks, n)):
        dev = torch.device("cuda", k)
        with torch.cuda.device(dev):
            data, offsets, _ = _data(torch, dev, chunk_range=(lo, hi))
            st = torch.cuda.current_stream(dev).cuda_stream
        c = get_context(k)
        plans.append(ReductionPlan(c, np.float32, (64, 64, 64), data.data_ptr(), offsets, missing=MISSING,
                                   stream=st))
        ctxs.append(c)
        streams.append(st)
        keep.append(data)
    res = _sharded(ctxs, plans, streams)
    dev0 = torch.device("cuda", 0)
    data, offsets, _ = _data(torch, dev0)
    st0 = torch.cuda.current_stream(dev0).cuda_stream
    one = ReductionPlan(gpu, np.float32, (64, 64, 64), data.data_ptr(), offsets, missing=MISSING, stream=st0)
    one.launch(st0, chunk_partials=False)
    want = one.read_total(st0)[0]
    for r in res:
        assert r[0].tobytes() == res[0][0].tobytes()      # every device holds the same total
        g = r[0]
        assert g["count"] == want["count"] and g["min"] == want["min"] and g["max"] == want["max"]
        assert abs(g["sum"] - want["sum"]) <= 1e-6 * abs(want["sum"])
