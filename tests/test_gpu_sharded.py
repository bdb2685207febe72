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
SHAPE, CHUNKS = (256, 128, 128), (64, 64, 64)


def _data(ctx, st, lo=0, hi=None):
    """Chunks [lo, hi) of a dummy_data-style variable with planted fill
    values, uploaded with the library's own copies (this process's HIP
    runtime belongs to libpyas_hip: no torch here)."""
    from pyactivestorage_amd.device import DeviceBuffer
    from pyactivestorage_amd.synthetic import chunk_major_host
    buf, offsets = chunk_major_host(SHAPE, CHUNKS, np.float32)
    vals = buf.view(np.float32).copy()
    vals[np.random.default_rng(5).random(vals.size) < 0.01] = -999.0
    cb = int(np.prod(CHUNKS)) * 4
    hi = len(offsets) if hi is None else hi
    part = vals.view(np.uint8)[lo * cb: hi * cb]
    d = DeviceBuffer(ctx, max(part.nbytes, 16))
    ctx.h2d(d.ptr, part, st)
    ctx.synchronize(st)
    return d, np.arange(hi - lo, dtype=np.int64) * cb


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
    st = gpu.thread_stream()
    data, offsets = _data(gpu, st)
    plan = ReductionPlan(gpu, np.float32, CHUNKS, data.ptr, offsets, missing=MISSING, stream=st)
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
    st = gpu.thread_stream()
    data, offsets = _data(gpu, st, 0, 4)
    plan = ReductionPlan(gpu, np.float32, CHUNKS, data.ptr, offsets, missing=MISSING, stream=st)
    out = DeviceBuffer(gpu, 3 * _lib.PARTIAL_NBYTES)
    rc = lib.pyas_reduce_sharded(_arr(ctypes.c_void_p, [gpu.handle, gpu.handle]),
                                 _arr(ctypes.c_void_p, [ctypes.addressof(plan.batch)] * 2), None, 2, 0,
                                 _arr(ctypes.c_void_p, [out.ptr, out.ptr]), _arr(ctypes.c_void_p, [st, st]))
    assert rc == _lib.EINVAL and b"appears twice" in lib.pyas_last_error()


def test_several_devices_equal_one(gpu):
    n = ctypes.c_int(0)
    _lib.check(gpu.lib.pyas_device_count(ctypes.byref(n)), "pyas_device_count")
    if n.value < 2:
        pytest.skip("one GPU visible: the ndev > 1 exchange runs on multi-GPU nodes only")
    from pyactivestorage_amd.distributed import equal_ranges
    n_chunks = int(np.prod([s // c for s, c in zip(SHAPE, CHUNKS)]))
    ctxs, plans, streams, keep = [], [], [], []
    for k, (lo, hi) in enumerate(equal_ranges(n_chunks, n.value)):
        c = get_context(k)
        st = c.thread_stream()
        data, offsets = _data(c, st, lo, hi)
        plans.append(ReductionPlan(c, np.float32, CHUNKS, data.ptr, offsets, missing=MISSING, stream=st))
        ctxs.append(c)
        streams.append(st)
        keep.append(data)
    res = _sharded(ctxs, plans, streams)
    st0 = gpu.thread_stream()
    data, offsets = _data(gpu, st0)
    one = ReductionPlan(gpu, np.float32, CHUNKS, data.ptr, offsets, missing=MISSING, stream=st0)
    one.launch(st0, chunk_partials=False)
    want = one.read_total(st0)[0]
    for r in res:
        assert r[0].tobytes() == res[0][0].tobytes()      # every device holds the same total
        g = r[0]
        assert g["count"] == want["count"] and g["min"] == want["min"] and g["max"] == want["max"]
        assert abs(g["sum"] - want["sum"]) <= 1e-6 * abs(want["sum"])


def test_bounded_wait(gpu, monkeypatch):
    """PYAS_SHARD_TIMEOUT_MS: with a deadline the call waits for the exchange;
    a zero deadline on a stream still busy with a long reduce returns
    PYAS_EDEVICE naming the device, and -- its collective queued but not
    started -- keeps the communicators (aborting would free them
    under the queued RCCL kernel); the exchange completes on the stream and
    the next call succeeds on the same communicators."""
    st = gpu.thread_stream()
    data, offsets = _data(gpu, st)
    plan = ReductionPlan(gpu, np.float32, CHUNKS, data.ptr, offsets, missing=MISSING, stream=st)
    plan.launch(st, chunk_partials=False)
    want = plan.read_total(st)
    monkeypatch.setenv("PYAS_SHARD_TIMEOUT_MS", "60000")
    got = _sharded([gpu], [plan], [st])[0]
    assert got[0].tobytes() == want.tobytes()
    # ~8 GiB of reads (the 32 chunks 256 times over) keep the stream busy
    big = ReductionPlan(gpu, np.float32, CHUNKS, data.ptr, np.tile(offsets, 256), missing=MISSING, stream=st)
    monkeypatch.setenv("PYAS_SHARD_TIMEOUT_MS", "0")
    n = 1
    outs = [DeviceBuffer(gpu, (n + 1) * _lib.PARTIAL_NBYTES)]
    lib = gpu.lib
    rc = lib.pyas_reduce_sharded(
        _arr(ctypes.c_void_p, [gpu.handle]), _arr(ctypes.c_void_p, [ctypes.addressof(big.batch)]),
        _arr(ctypes.c_void_p, [ctypes.addressof(big.mask_up.struct)]), n, 1,
        _arr(ctypes.c_void_p, [o.ptr for o in outs]), _arr(ctypes.c_void_p, [st]))
    gpu.synchronize(st)
    assert rc == _lib.EDEVICE, rc
    msg = lib.pyas_last_error()
    assert b"did not finish" in msg and b"device(s) %d" % gpu.device in msg, msg
    assert b"communicators were kept" in msg, msg
    host = np.zeros(n + 1, dtype=engine.partial_dtype(np.float32))
    gpu.d2h(host, outs[0].ptr, st)
    gpu.synchronize(st)
    assert host[1]["count"] == 256 * want["count"][0]   # the queued exchange delivered the total
    monkeypatch.delenv("PYAS_SHARD_TIMEOUT_MS")
    got = _sharded([gpu], [plan], [st])[0]
    assert got[0].tobytes() == want.tobytes()


def _sharded_tie(ctxs, plans, streams, which, geom, flags=1):
    n = len(ctxs)
    outs = [DeviceBuffer(c, (n + 1) * _lib.PARTIAL_NBYTES) for c in ctxs]
    lib = ctxs[0].lib
    rc = lib.pyas_reduce_sharded_tie(
        _arr(ctypes.c_void_p, [c.handle for c in ctxs]),
        _arr(ctypes.c_void_p, [ctypes.addressof(p.batch) for p in plans]),
        _arr(ctypes.c_void_p, [ctypes.addressof(p.mask_up.struct) for p in plans]),
        n, flags, ctypes.addressof(geom), which, _arr(ctypes.c_void_p, [o.ptr for o in outs]),
        _arr(ctypes.c_void_p, streams))
    _lib.check(rc, "pyas_reduce_sharded_tie")
    res = []
    for c, o, s, p in zip(ctxs, outs, streams, plans):
        host = np.zeros(n + 1, dtype=engine.partial_dtype(p.dtype))
        c.d2h(host, o.ptr, s)
        c.synchronize(s)
        res.append(host)
    return res


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("kind", ["min", "max"])
@pytest.mark.parametrize("dens", [0.2, 0.002])
def test_sharded_zero_sign(gpu, dt, kind, dens):
    """pyas_reduce_sharded_tie gives a zero min/max NumPy's
    sign (storage.py:99-100 per chunk, active.py:594 over the per-chunk
    results), byte for byte against the oracle's reduce_chunk composed as
    active.py does; at ndev = 1 here, and split over every visible GPU on a
    multi-GPU node.  Without the sign (pyas_reduce_sharded) the value and
    count are the same."""
    from tests.test_gpu_zero_sign import _chunk, _reference_active, _variable
    from pyactivestorage_amd.distributed import equal_ranges
    from pyactivestorage_amd.zerosign import tie_rule
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(11 + len(kind) + int(dens * 1000) + len(dt))
    shape, chunks = (16, 24, 80), (4, 8, 20)
    a = _chunk(rng, shape, np.dtype(dt), "min0" if kind == "min" else "max0", dens=dens, n_fill=10)
    missing = (np.dtype(dt).type(-999.0), None, None, None)
    var, data = _variable(a, chunks, {"_FillValue": np.array([-999.0], dtype=dt)})
    data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
    want = _reference_active(a, chunks, (slice(None),) * 3, (0, 1, 2), kind, missing, data_of)
    wv = np.ma.getdata(want).reshape(-1)[0]
    assert wv == 0                                    # the case the sign matters for
    n = ctypes.c_int(0)
    _lib.check(gpu.lib.pyas_device_count(ctypes.byref(n)), "pyas_device_count")
    cb = int(np.prod(chunks)) * np.dtype(dt).itemsize
    n_chunks = len(var.chunk_index)
    host = np.frombuffer(data, dtype=np.uint8)
    ctxs, plans, streams, keep = [], [], [], []
    for k, (lo, hi) in enumerate(equal_ranges(n_chunks, max(1, n.value))):
        c = get_context(k)
        st = c.thread_stream()
        d = DeviceBuffer(c, max((hi - lo) * cb, 16))
        c.h2d(d.ptr, host[lo * cb: hi * cb], st)
        c.synchronize(st)
        plans.append(ReductionPlan(c, np.dtype(dt), chunks, d.ptr, np.arange(hi - lo, dtype=np.int64) * cb,
                                   missing=missing, stream=st))
        ctxs.append(c)
        streams.append(st)
        keep.append(d)
    which = 1 if kind == "min" else 2
    got = _sharded_tie(ctxs, plans, streams, which, plans[0].tie_geom())
    plain = _sharded(ctxs, plans, streams) if dt == "<f4" else None
    for r in got:
        g = r[0][kind]
        assert g == wv and np.signbit(g) == np.signbit(wv), (kind, dens, g, wv)
        assert r[0].tobytes() == got[0][0].tobytes()
        if plain is not None:
            assert r[0]["count"] == plain[0][0]["count"] and r[0][kind] == plain[0][0][kind]
