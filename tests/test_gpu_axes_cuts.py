"""Partial-axis reductions of cut chunks in the dense kernels, against the oracle.

A hyperslab's edge chunks are cut boxes (unit steps).  When the box covers at
least half the chunk, the dense kernels (column layout, row layout, LDS row
layout) read the cut chunk as a whole one: reduced positions outside the box
are excluded (a per-row bit map in LDS for the column walks, per-element bits
for the row layouts) and only the outputs inside the box are written, each at
its place in the chunk's partial array (``cut_eligible`` / ``cut_map`` /
``cut_out`` in pyas_kernels.hpp).  Thinner boxes stay on ``k_reduce_axes``.

Each case runs one ``pyas_reduce_axes`` call over a batch mixing whole
chunks, cut boxes at either end of one, two or every dim (the shapes of
``[1:1023]``-style hyperslab edges), boxes just above and below the half-chunk
rule, and element- but not 16-byte-aligned chunk offsets; every chunk's
partials (count, sum, min, max per output) are compared with
``oracle.storage_ref.reduce_chunk_bytes`` (``storage.py:95-100``): count,
min and max exact, sums within 1e-6.  ``PYAS_AXES_CUTS=0`` (every cut chunk
on the generic walk) must give the same counts/min/max.
Template: ``tests/unit/test_active_axis.py:30-78`` (hyperslabs x axis subsets).
"""
import itertools
import os

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import _lib, engine, selection
from tests._compare import shuffle_bytes

pytestmark = pytest.mark.gpu


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


def _boxes(shape, rng):
    """Whole chunk, edge cuts (1 from either end of 1, 2 and all dims), a
    ragged interior box, and boxes either side of the half-chunk rule."""
    nd = len(shape)
    full = tuple(slice(0, n) for n in shape)
    out = [full]
    for k in (1, 2, nd):
        for dims in list(itertools.combinations(range(nd), min(k, nd)))[:3]:
            for lo_side in (True, False):
                b = list(full)
                for d in dims:
                    b[d] = slice(1, shape[d]) if lo_side else slice(0, shape[d] - 1)
                out.append(tuple(b))
    b = [slice(int(rng.integers(0, max(1, n // 8))), n - int(rng.integers(0, max(1, n // 8)))) for n in shape]
    out.append(tuple(b))
    # about half the chunk along dim 0 (one above the rule, one below)
    n0 = shape[0]
    out.append((slice(0, n0 // 2 + (1 if n0 % 2 else 0)),) + full[1:])
    if n0 >= 4:
        out.append((slice(1, n0 // 2),) + full[1:])
    return out


def _axes(nd):
    out = []
    for k in range(1, nd):
        out += list(itertools.combinations(range(nd), k))
    return out


CASES = [("<f4", (8, 16, 32)), ("<f4", (4, 4, 64)), (">f8", (6, 8, 16)), ("<i2", (8, 8, 32)),
         ("<f4", (4, 6, 4, 16)), ("u1", (4, 8, 64)), ("<i8", (4, 8, 16))]


def _run(ctx, dt, shape, shuf, axes, miss, boxes, chunks):
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import DeviceBuffer
    es = dt.itemsize
    st = ctx.thread_stream()
    n = len(chunks)
    cbytes = chunks[0].nbytes
    offsets = np.array([k * (cbytes + es) + es for k in range(n)], dtype=np.int64)
    blob = np.zeros(int(offsets[-1]) + cbytes + 16, dtype=np.uint8)
    for k, a in enumerate(chunks):
        raw = shuffle_bytes(a, es) if shuf else a.tobytes()
        blob[offsets[k]:offsets[k] + cbytes] = np.frombuffer(raw, np.uint8)
    dbuf = DeviceBuffer(ctx, blob.nbytes)
    ctx.h2d(dbuf.ptr, blob, st)
    csels = [selection.normalize(b, shape) for b in boxes]
    plan = ReductionPlan(ctx, dt, shape, dbuf.ptr, offsets, selections=csels, missing=miss, stream=st,
                         shuffle=es if shuf else 0)
    n_outs = [int(np.prod([1 if d in axes else c.shape[d] for d in range(len(shape))])) for c in csels]
    out_offs = np.concatenate([[0], np.cumsum(n_outs)[:-1]]).astype(np.int64)
    offs_t = DeviceBuffer(ctx, out_offs.nbytes)
    ctx.h2d(offs_t.ptr, out_offs, st)
    out = DeviceBuffer(ctx, int(sum(n_outs)) * _lib.PARTIAL_NBYTES)
    engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, sum(1 << a for a in axes), offs_t.ptr, out.ptr, st)
    host = np.zeros(int(sum(n_outs)), dtype=engine.partial_dtype(dt))
    ctx.d2h(host, out.ptr, st)
    ctx.synchronize(st)
    for b in (dbuf, offs_t, out):
        b.free()
    return [host[out_offs[k]:out_offs[k] + n_outs[k]] for k in range(n)]


def _check(dt, chunks, boxes, axes, miss, parts, what):
    nd_dt = dt.newbyteorder("=")
    for k, a in enumerate(chunks):
        vals, _ = ref.reduce_chunk_bytes(a.tobytes(), None, None, miss, dt.str, a.shape, "C", boxes[k], axes, None)
        m = np.ma.getmaskarray(vals)
        v = np.ma.getdata(vals)
        cnt = (~m).sum(axis=axes, keepdims=True).reshape(-1)
        p = parts[k]
        w = f"{what} chunk {k} box {boxes[k]}"
        np.testing.assert_array_equal(p["count"], cnt, err_msg=w)
        ok = cnt > 0
        vm = np.ma.MaskedArray(v.astype(nd_dt), mask=m)
        wmin = np.ma.getdata(np.ma.min(vm, axis=axes, keepdims=True)).reshape(-1)
        wmax = np.ma.getdata(np.ma.max(vm, axis=axes, keepdims=True)).reshape(-1)
        np.testing.assert_array_equal(p["min"][ok].astype(nd_dt), wmin[ok], err_msg=w)
        np.testing.assert_array_equal(p["max"][ok].astype(nd_dt), wmax[ok], err_msg=w)
        acc = np.float64 if dt.kind == "f" else (np.int64 if dt.kind == "i" else np.uint64)
        wsum = np.ma.filled(vm.astype(acc), 0).sum(axis=axes, keepdims=True).reshape(-1)
        if dt.kind == "f":
            np.testing.assert_allclose(p["sum"][ok], wsum[ok], rtol=1e-6, atol=1e-3, err_msg=w)
        else:
            np.testing.assert_array_equal(p["sum"][ok], wsum[ok], err_msg=w)


@pytest.mark.parametrize("shuf", [False, True])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("case", range(len(CASES)), ids=[f"{d}-{'x'.join(map(str, s))}" for d, s in CASES])
def test_cut_chunks_match_oracle(gpu, case, masked, shuf):
    dt, shape = CASES[case]
    dt = np.dtype(dt)
    if shuf and dt.itemsize == 1:
        pytest.skip("shuffle is the identity for 1-byte types")
    rng = np.random.default_rng(case * 4 + 2 * masked + shuf)
    boxes = _boxes(shape, rng)
    chunks = [_data(dt, shape, rng, nan=(k == 3 and dt.kind == "f")) for k in range(len(boxes))]
    miss = (42, None, 0, 90) if masked else (None, None, None, None)
    for axes in _axes(len(shape)):
        parts = _run(gpu, dt, shape, shuf, axes, miss, boxes, chunks)
        _check(dt, chunks, boxes, axes, miss, parts, f"{dt} {shape} shuf={shuf} masked={masked} axes={axes}")


@pytest.mark.parametrize("axes", [(0,), (2,), (1,), (0, 1), (1, 2)])
def test_cuts_off_agrees(gpu, axes, monkeypatch):
    """PYAS_AXES_CUTS=0 (every cut chunk on k_reduce_axes) and the dense cut
    path give the same counts, minima and maxima, byte for byte."""
    dt, shape = np.dtype("<f4"), (16, 16, 64)
    rng = np.random.default_rng(3)
    boxes = _boxes(shape, rng)
    chunks = [_data(dt, shape, rng) for _ in boxes]
    miss = (42, None, 0, 90)
    on = _run(gpu, dt, shape, False, axes, miss, boxes, chunks)
    monkeypatch.setenv("PYAS_AXES_CUTS", "0")
    off = _run(gpu, dt, shape, False, axes, miss, boxes, chunks)
    for a, b in zip(on, off):
        assert a["count"].tobytes() == b["count"].tobytes()
        assert a["min"].tobytes() == b["min"].tobytes()
        assert a["max"].tobytes() == b["max"].tobytes()
        np.testing.assert_allclose(a["sum"], b["sum"], rtol=1e-6)
