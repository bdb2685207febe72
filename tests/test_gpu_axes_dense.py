"""GPU parity of the dense partial-axis kernels (``k_axes_dense``) against
the oracle.

The dense kernels take fully selected chunks (plain or HDF5-shuffled: the
shuffled form loads each 16-B vector as one piece per byte plane) whose merged dims
fit (RO, KO, RI, KI) with 16-byte inner runs (column layout: kept inner run;
row layout: reduced inner run, including the 4-outputs-per-lane variant).
The reference semantics are ``storage.py:95-100`` (``chunk[sel]``, mask,
``method(axis, keepdims=True)``, ``np.ma.count``) and the sweep mirrors
``tests/unit/test_active_axis.py:30-78`` (every axis subset x methods).
Shapes are chosen so every layout and fallback is hit; the batch test mixes
fully and partially selected chunks in one call (both kernels run, each
skipping the other's chunks) at element- but not 16-byte-aligned offsets.
"""
import itertools

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import _lib, engine
from pyactivestorage_amd import storage as pas
from tests._compare import assert_counts, assert_same, shuffle_bytes

pytestmark = pytest.mark.gpu

DTYPES = ["<f4", ">f4", "<f8", ">f8", "<i2", "<i4", ">u4", "<i8", "i1", "u1"]
# (8,16,32): every layout; (2,4,64): column with few items, row with 4
# outputs per lane; (4,4,4,16): 4-D patterns incl. R K R K; (3,5,8): rows of
# 8 elements (row layout with G < 4 for f4 -> generic fallback)
SHAPES = [(8, 16, 32), (2, 4, 64), (4, 4, 4, 16), (3, 5, 8)]
METHODS = [np.ma.sum, np.ma.min, np.ma.max, np.ma.mean]


def _data(dt, shape, rng, nan=False):
    dt = np.dtype(dt)
    if dt.kind == "f":
        a = rng.uniform(-50, 150, size=shape).astype(dt)
        a.reshape(-1)[::13] = 42.0
        if nan:
            a.reshape(-1)[5] = np.nan
    else:
        info = np.iinfo(dt)
        a = rng.integers(max(info.min, -100), min(info.max, 100), size=shape, endpoint=True).astype(dt)
        a.reshape(-1)[::13] = 42
    return a


def _missings(dt):
    return [(None, None, None, None), (42, None, 0, 90), (None, None, None, -1e30)]


def _axes(ndim):
    out = []
    for k in range(1, ndim):
        out += list(itertools.combinations(range(ndim), k))
    return out


def _cases():
    out = []
    for dt in DTYPES:
        for shape in SHAPES:
            for mi, miss in enumerate(_missings(dt)):
                out.append((dt, shape, mi))
    return out


CASES = _cases()


@pytest.mark.parametrize("shuf", [False, True])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_dense_chunk_matches_oracle(gpu, case, shuf):
    dt, shape, mi = CASES[case]
    miss = _missings(dt)[mi]
    rng = np.random.default_rng(case)
    arr = _data(dt, shape, rng, nan=(case % 4 == 0))
    es = np.dtype(dt).itemsize
    raw = shuffle_bytes(arr, es) if shuf else arr.tobytes()
    rf = [ref.Shuffle(es)] if shuf else None
    gf = [pas.Shuffle(es)] if shuf else None
    sel = tuple(slice(0, n, 1) for n in shape)
    for axis in _axes(len(shape)):
        for method in METHODS:
            what = f"{dt} {shape} shuf={shuf} miss={miss} axis={axis} {method.__name__}"
            want, wn = ref.reduce_chunk_bytes(raw, None, rf, miss, dt, shape, "C", sel, axis, method)
            got, gn = pas.reduce_chunk_bytes(raw, None, gf, miss, dt, shape, "C", sel, axis, method)
            masked_sel, _ = ref.reduce_chunk_bytes(raw, None, rf, miss, dt, shape, "C", sel, axis, None)
            with np.errstate(all="ignore"):
                abs_sum = np.ma.sum(np.abs(np.ma.asarray(masked_sel).astype(np.float64)),
                                    axis=axis, keepdims=True)
            assert_same(want, got, method.__name__, np.ma.filled(abs_sum, 0), what)
            assert_counts(wn, gn, what)


def _oracle_partials(arr, sel, axis, miss, dt):
    """Per-output {sum, count, min, max} of one chunk from the oracle."""
    raw = arr.tobytes()
    shape = arr.shape
    vals, _ = ref.reduce_chunk_bytes(raw, None, None, miss, dt, shape, "C", sel, axis, None)
    m = np.ma.getmaskarray(vals)
    v = np.ma.getdata(vals)
    cnt = (~m).sum(axis=axis, keepdims=True).reshape(-1)
    return v, m, cnt


@pytest.mark.parametrize("shuf", [False, True])
@pytest.mark.parametrize("dt", ["<f4", ">f8", "<i2", "<u8"])
@pytest.mark.parametrize("axes", [(0,), (2,), (1, 2), (0, 2)])
def test_dense_batch_mixed_and_misaligned(gpu, dt, axes, shuf):
    """One pyas_reduce_axes call over 6 chunks: full and hyperslab selections
    interleaved, chunk offsets at element (not 16-byte) alignment; shuffled:
    <i2 chunks are not 8-byte aligned, so their plane pieces take the
    unaligned loads."""
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import DeviceBuffer, get_context
    dt = np.dtype(dt)
    es = dt.itemsize
    shape = (8, 16, 32)
    ctx = get_context(0)
    st = ctx.thread_stream()
    rng = np.random.default_rng(11)
    chunks = [_data(dt, shape, rng, nan=(k == 2)) for k in range(6)]
    full = tuple(slice(0, n, 1) for n in shape)
    part = (slice(1, 7, 1), slice(0, 16, 1), slice(2, 30, 1))
    sels = [full, part, full, full, part, full]
    cbytes = chunks[0].nbytes
    offsets = np.array([k * (cbytes + es) + es for k in range(6)], dtype=np.int64)
    blob = np.zeros(int(offsets[-1]) + cbytes + 16, dtype=np.uint8)
    for k, a in enumerate(chunks):
        raw = shuffle_bytes(a, es) if shuf else a.tobytes()
        blob[offsets[k]:offsets[k] + cbytes] = np.frombuffer(raw, np.uint8)
    dbuf = DeviceBuffer(ctx, blob.nbytes)
    ctx.h2d(dbuf.ptr, blob, st)
    miss = (42, None, 0, 90)
    from pyactivestorage_amd import selection
    csels = [selection.normalize(s, shape) for s in sels]
    plan = ReductionPlan(ctx, dt, shape, dbuf.ptr, offsets,
                         selections=[selection.ChunkSel(c.dims, c.shape, c.kept) for c in csels],
                         missing=miss, stream=st, shuffle=es if shuf else 0)
    n_outs = [int(np.prod([1 if d in axes else c.shape[d] for d in range(3)])) for c in csels]
    out_offs = np.concatenate([[0], np.cumsum(n_outs)[:-1]]).astype(np.int64)
    offs_t = DeviceBuffer(ctx, out_offs.nbytes)
    ctx.h2d(offs_t.ptr, out_offs, st)
    out = DeviceBuffer(ctx, int(sum(n_outs)) * _lib.PARTIAL_NBYTES)
    mask_bits = sum(1 << a for a in axes)
    engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, mask_bits, offs_t.ptr, out.ptr, st)
    host = np.zeros(int(sum(n_outs)), dtype=engine.partial_dtype(dt))
    ctx.d2h(host, out.ptr, st)
    ctx.synchronize(st)
    nd = dt.newbyteorder("=")
    for k, a in enumerate(chunks):
        part_k = host[out_offs[k]:out_offs[k] + n_outs[k]]
        v, m, cnt = _oracle_partials(a, sels[k], axes, miss, dt)
        what = f"{dt} axes={axes} chunk {k}"
        np.testing.assert_array_equal(part_k["count"], cnt, err_msg=what)
        ok = cnt > 0
        vm = np.ma.MaskedArray(v.astype(nd), mask=m)
        wmin = np.ma.getdata(np.ma.min(vm, axis=axes, keepdims=True)).reshape(-1)
        wmax = np.ma.getdata(np.ma.max(vm, axis=axes, keepdims=True)).reshape(-1)
        np.testing.assert_array_equal(part_k["min"][ok].astype(nd), wmin[ok], err_msg=what)
        np.testing.assert_array_equal(part_k["max"][ok].astype(nd), wmax[ok], err_msg=what)
        acc = np.float64 if dt.kind == "f" else (np.int64 if dt.kind == "i" else np.uint64)
        wsum = np.ma.filled(vm.astype(acc), 0).sum(axis=axes, keepdims=True).reshape(-1)
        if dt.kind == "f":
            np.testing.assert_allclose(part_k["sum"][ok], wsum[ok], rtol=1e-6, atol=1e-3, err_msg=what)
        else:
            np.testing.assert_array_equal(part_k["sum"][ok], wsum[ok], err_msg=what)


@pytest.mark.parametrize("with_sels", [True, False])
def test_vector_fill_on_whole_chunks(gpu, with_sels):
    """Broadcast (vector) missing values on fully selected chunks: the
    selection table may not be dropped (the lean kernel applies scalar rules
    only) and a NULL table must still route to the table-aware kernel.
    Reference: storage.py:133-143 (broadcast ==)."""
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import DeviceBuffer, get_context
    from pyactivestorage_amd import selection
    dt = np.dtype("<f4")
    shape = (4, 6, 8)
    ctx = get_context(0)
    st = ctx.thread_stream()
    rng = np.random.default_rng(5)
    chunks = [_data(dt, shape, rng) for _ in range(5)]
    vec = np.arange(8, dtype=np.float32) + 40.0           # broadcast along the last dim
    for a in chunks:
        a[..., 2] = 42.0                                  # matches vec[2]
    miss = (None, vec, None, None)
    blob = np.concatenate([np.frombuffer(a.tobytes(), np.uint8) for a in chunks])
    dbuf = DeviceBuffer(ctx, blob.nbytes)
    ctx.h2d(dbuf.ptr, blob, st)
    offsets = np.arange(5, dtype=np.int64) * chunks[0].nbytes
    full = tuple(slice(0, n, 1) for n in shape)
    sels = [selection.normalize(full, shape) for _ in chunks] if with_sels else None
    plan = ReductionPlan(ctx, dt, shape, dbuf.ptr, offsets, selections=sels, missing=miss,
                         round_to_var=False, stream=st)
    plan.launch(st)
    tot = plan.read_total(st)[0]
    want_n, want_sum, mins, maxs = 0, 0.0, [], []
    for a in chunks:
        m, n = ref.reduce_chunk_bytes(a.tobytes(), None, None, miss, dt, shape, "C", full,
                                      (0, 1, 2), np.ma.sum)
        want_n += int(np.asarray(n).reshape(-1)[0])
        want_sum += float(np.ma.filled(m, 0).reshape(-1)[0])
        mins.append(float(np.ma.min(ref.reduce_chunk_bytes(a.tobytes(), None, None, miss, dt, shape, "C",
                                                            full, (0, 1, 2), None)[0])))
        maxs.append(float(np.ma.max(ref.reduce_chunk_bytes(a.tobytes(), None, None, miss, dt, shape, "C",
                                                            full, (0, 1, 2), None)[0])))
    assert int(tot["count"]) == want_n and want_n < 5 * chunks[0].size
    assert float(tot["min"]) == min(mins) and float(tot["max"]) == max(maxs)
    np.testing.assert_allclose(float(tot["sum"]), want_sum, rtol=1e-6)
