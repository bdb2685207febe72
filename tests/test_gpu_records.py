"""Compact per-output records of the partial-axis reduction
(``pyas_reduce_axes_ex``, pyas.h ``PYAS_REC_*``).

Per chunk, ``storage.reduce_chunk`` returns one method's result and the count
(``activestorage/storage.py:98-104``), and ``Active`` stores it in an ``out``
array of the variable dtype (``active.py:512,585``).  The records carry just
that: the sum rounded to the variable dtype (integer sums wrapped), or the
min, or the max, plus an int32 count -- 8 bytes per output for 1/2/4-byte
dtypes instead of the 32-byte partial.  Every per-chunk kernel writes them
(column, streamed column, butterfly row, LDS row, and the generic kernel of
hyperslab/list selections); each is forced here through the library's
layout switches, and every record must equal the 32-byte partial of the same
launch converted on the host, byte for byte (value, count, sign of a zero,
NaN).  The combines and zero-sign passes that read records are covered
end to end by the Active tests (their two-step path uses records).
"""
import numpy as np
import pytest

from pyactivestorage_amd import _lib, engine, selection
from tests._compare import assert_partials_match_oracle, oracle_partials, shuffle_bytes

pytestmark = pytest.mark.gpu

# (shape, axes, env): geometries that route to each per-chunk kernel
LAYOUTS = [
    ((8, 32, 64), (0,), {"PYAS_COL_STREAM": "0"}),          # dense_col
    ((8, 64, 64), (0,), {"PYAS_COL_STREAM": "3"}),          # k_axes_col_stream, ragged last workgroup
    ((16, 8, 128), (1,), {}),                               # column layout, host's choice
    ((8, 16, 64), (2,), {"PYAS_ROW_LDS": "2"}),             # dense_row_lds
    ((8, 16, 64), (2,), {"PYAS_ROW_LDS": "0"}),             # butterfly row layout
    ((4, 8, 512), (1, 2), {}),                              # row layout, long runs
    ((6, 10, 14), (0, 2), {}),                              # odd extents
]
DTYPES = ["<f4", ">f4", "<f8", "<i2", "<u1", "<i4", "<i8"]


def _chunks(dt, shape, n, rng):
    out = []
    for k in range(n):
        if dt.kind == "f":
            a = rng.uniform(-60, 150, size=shape).astype(dt)
            a.reshape(-1)[rng.random(a.size) < 0.05] = -999
            a.reshape(-1)[rng.random(a.size) < 0.03] = 0.0
            a.reshape(-1)[rng.random(a.size) < 0.03] = -0.0
            if k == 1:
                a.reshape(-1)[rng.integers(0, a.size, 2)] = np.nan
        else:
            info = np.iinfo(dt)
            a = rng.integers(max(info.min, -30000), min(info.max, 30000), size=shape, endpoint=True).astype(dt)
        out.append(a)
    return out


def _expected(full, dt, rec):
    """Host conversion of 32-byte partials to records (pyas.h PYAS_REC_*)."""
    nd = dt.newbyteorder("=")
    n = full.size
    rb = _lib.rec_nbytes(dt.itemsize, rec)
    out = np.zeros((n, rb), dtype=np.uint8)
    if rec == _lib.REC_SUM:
        with np.errstate(over="ignore", invalid="ignore"):
            vals = full["sum"].astype(nd) if dt.kind == "f" else full["sum"].astype(np.int64).astype(nd)
    else:
        vals = full["min" if rec == _lib.REC_MIN else "max"].astype(nd)
    out[:, :dt.itemsize] = np.ascontiguousarray(vals).view(np.uint8).reshape(n, dt.itemsize)
    c0 = 4 if dt.itemsize <= 4 else 8
    out[:, c0:c0 + 4] = full["count"].astype("<i4").view(np.uint8).reshape(n, 4)
    return out


def _run(ctx, st, plan, axes_bits, out_offs, n_total, dt, rec):
    from pyactivestorage_amd.device import DeviceBuffer
    offs = DeviceBuffer(ctx, out_offs.nbytes)
    ctx.h2d(offs.ptr, out_offs, st)
    rb = _lib.rec_nbytes(dt.itemsize, rec)
    out = DeviceBuffer(ctx, max(n_total, 1) * rb)
    engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, axes_bits, offs.ptr, out.ptr, st, rec=rec)
    host = np.zeros(n_total * rb, dtype=np.uint8)
    ctx.d2h(host, out.ptr, st)
    ctx.synchronize(st)
    return host


def _same_records(got, want, dt, what):
    got = got.reshape(want.shape)
    n = want.shape[0]
    c0 = 4 if dt.itemsize <= 4 else 8
    assert np.array_equal(got[:, c0:], want[:, c0:]), (what, "count")
    nd = dt.newbyteorder("=")
    gv = got[:, :dt.itemsize].copy().view(nd).reshape(n)
    wv = want[:, :dt.itemsize].copy().view(nd).reshape(n)
    if dt.kind == "f":
        nan = np.isnan(wv)
        assert np.array_equal(nan, np.isnan(gv)), (what, "nan")
        assert gv[~nan].tobytes() == wv[~nan].tobytes(), (what, gv[~nan][gv[~nan] != wv[~nan]][:5])
    else:
        assert np.array_equal(gv, wv), what
    assert not got[:, dt.itemsize:c0].any(), (what, "padding")


@pytest.mark.parametrize("layout", range(len(LAYOUTS)))
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shuf", [False, True])
@pytest.mark.parametrize("sel", ["whole", "hyperslab"])
def test_records_equal_converted_partials(gpu, layout, dtype, shuf, sel, monkeypatch):
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import DeviceBuffer
    shape, axes, env = LAYOUTS[layout]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    dt = np.dtype(dtype)
    es = dt.itemsize
    if shuf and es == 1:
        pytest.skip("a 1-byte shuffle is the identity")
    rng = np.random.default_rng(layout * 31 + len(dtype) + shuf)
    n = 7
    chunks = _chunks(dt, shape, n, rng)
    cbytes = chunks[0].nbytes
    offsets = np.arange(n, dtype=np.int64) * (cbytes + 256)
    blob = np.zeros(int(offsets[-1]) + cbytes + 16, dtype=np.uint8)
    for k, a in enumerate(chunks):
        raw = shuffle_bytes(a, es) if shuf else a.tobytes()
        blob[offsets[k]:offsets[k] + cbytes] = np.frombuffer(raw, np.uint8)
    ctx, st = gpu, gpu.thread_stream()
    dbuf = DeviceBuffer(ctx, blob.nbytes)
    ctx.h2d(dbuf.ptr, blob, st)
    miss = (dt.type(-999), None, None, None) if dt.kind == "f" else None
    sels = None
    if sel == "hyperslab":
        full = tuple(slice(0, m, 1) for m in shape)
        cut = tuple(slice(1, m - 1, 1) if m > 4 else slice(0, m, 1) for m in shape)
        sels = [selection.normalize(full if k % 2 == 0 else cut, shape) for k in range(n)]
    plan = ReductionPlan(ctx, dt, shape, dbuf.ptr, offsets, selections=sels, missing=miss, stream=st,
                         shuffle=es if shuf else 0)
    cshape = [s.shape for s in sels] if sels else [shape] * n
    n_outs = [int(np.prod([1 if d in axes else cs[d] for d in range(len(shape))])) for cs in cshape]
    out_offs = np.concatenate([[0], np.cumsum(n_outs)[:-1]]).astype(np.int64)
    n_total = int(sum(n_outs))
    bits = sum(1 << a for a in axes)
    full_bytes = _run(ctx, st, plan, bits, out_offs, n_total, dt, _lib.REC_FULL)
    full = full_bytes.view(engine.partial_dtype(dt))
    assert int(full["count"].sum()) > 0
    for rec in (_lib.REC_SUM, _lib.REC_MIN, _lib.REC_MAX):
        got = _run(ctx, st, plan, bits, out_offs, n_total, dt, rec)
        _same_records(got, _expected(full, dt, rec), dt, (dtype, shape, axes, env, shuf, sel, rec))
    # the partials behind the records, straight against the oracle
    # (VERDICT r4 #7): the first chunk (whole) and the second (cut if hyperslab)
    for k in (0, 1):
        sk = tuple(slice(0, m) for m in shape) if sels is None else \
            tuple(slice(d.start, d.start + d.count) for d in sels[k].dims)
        assert_partials_match_oracle(full[out_offs[k]:out_offs[k] + n_outs[k]],
                                     oracle_partials(chunks[k], sk, axes, miss), dt,
                                     f"{dtype} {shape} axes={axes} {env} shuf={shuf} {sel} chunk {k}")


def test_record_argument_errors(gpu):
    lib = gpu.lib
    assert lib.pyas_reduce_axes_ex(gpu.handle, None, None, 1, 7, None, None, None) == _lib.EINVAL
