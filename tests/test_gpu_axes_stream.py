"""``k_axes_col_stream`` (per-chunk partial-axis reduce, column layout, each
workgroup walking several whole chunks as one ring of loads) against the
per-chunk ``dense_col`` walk it replaces, byte for byte, and against the
oracle.

The per-chunk partials are what ``storage.reduce_chunk`` returns for an axis
subset (``activestorage/storage.py:95-104``: ``method(chunk, axis,
keepdims=True)`` and ``np.ma.count``) before ``Active._from_storage`` folds
them (``activestorage/active.py:575-598``).  ``PYAS_COL_STREAM`` forces the
chunks per workgroup (0 = the per-chunk kernel), so small batches cover
ragged last workgroups (chunks not a multiple of cpb), cpb above the batch,
NaN, masked and unmasked modes, byte-swapped and shuffled chunks, and chunk
offsets that are not 16-byte aligned (the kernel's per-chunk fallback).
"""
import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import _lib, engine
from tests._compare import shuffle_bytes

pytestmark = pytest.mark.gpu

# (shape, axes): shapes whose column layout has >= 256 items per chunk
# (one lane per item column, split 1) and rows in whole 4-row groups.
# Plain f4 chunks of (8, 64, 64) / (4, 5, 1024) over (0,) take 4 items per
# lane (the second with a ragged last workgroup), the others 2 (f8 ones
# with item sets left empty); shuffled chunks take 1.
GEOMS = [((8, 32, 64), (0,)), ((16, 8, 128), (1,)), ((4, 4, 1024), (0, 1)), ((12, 16, 64), (0,)),
         ((8, 64, 64), (0,)), ((4, 5, 1024), (0,))]
DTYPES = ["<f4", ">f4", "<f8", "<i4", "<u8"]
MISSING = [None, (-999, None, -50, 140), (None, None, -1e30, None)]


def _chunks(dt, shape, n, rng, nan):
    out = []
    for k in range(n):
        if dt.kind == "f":
            a = rng.uniform(-60, 150, size=shape).astype(dt)
            a.reshape(-1)[rng.random(a.size) < 0.05] = -999
            a.reshape(-1)[rng.random(a.size) < 0.02] = 0.0
            a.reshape(-1)[rng.random(a.size) < 0.02] = -0.0
            if nan and k % 3 == 1:
                a.reshape(-1)[rng.integers(0, a.size, 2)] = np.nan
        else:
            lo = -1000 if dt.kind == "i" else 0
            a = rng.integers(lo, 1000, size=shape).astype(dt)
        out.append(a)
    return out


def _partials(ctx, st, dt, shape, chunks, axes, miss, shuf, misalign, stream_env, monkeypatch):
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import DeviceBuffer
    es = dt.itemsize
    cbytes = chunks[0].nbytes
    pad = es if misalign else 0
    offsets = np.array([k * (cbytes + 16 + pad) + pad for k in range(len(chunks))], dtype=np.int64)
    blob = np.zeros(int(offsets[-1]) + cbytes + 16, dtype=np.uint8)
    for k, a in enumerate(chunks):
        raw = shuffle_bytes(a, es) if shuf else a.tobytes()
        blob[offsets[k]:offsets[k] + cbytes] = np.frombuffer(raw, np.uint8)
    dbuf = DeviceBuffer(ctx, blob.nbytes)
    ctx.h2d(dbuf.ptr, blob, st)
    plan = ReductionPlan(ctx, dt, shape, dbuf.ptr, offsets, missing=miss, stream=st,
                         shuffle=es if shuf else 0)
    n_out = int(np.prod([1 if d in axes else shape[d] for d in range(len(shape))]))
    out_offs = np.arange(len(chunks), dtype=np.int64) * n_out
    offs = DeviceBuffer(ctx, out_offs.nbytes)
    ctx.h2d(offs.ptr, out_offs, st)
    out = DeviceBuffer(ctx, len(chunks) * n_out * _lib.PARTIAL_NBYTES)
    monkeypatch.setenv("PYAS_COL_STREAM", str(stream_env))
    engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, sum(1 << a for a in axes), offs.ptr, out.ptr, st)
    host = np.zeros(len(chunks) * n_out, dtype=engine.partial_dtype(dt))
    ctx.d2h(host, out.ptr, st)
    ctx.synchronize(st)
    return host.reshape(len(chunks), n_out)


@pytest.mark.parametrize("misalign", [False, True])
@pytest.mark.parametrize("shuf", [False, True])
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("geom", range(len(GEOMS)))
def test_stream_equals_per_chunk_walk(gpu, monkeypatch, geom, dt, shuf, misalign):
    from pyactivestorage_amd.device import get_context
    shape, axes = GEOMS[geom]
    dt = np.dtype(dt)
    ctx = get_context(0)
    st = ctx.thread_stream()
    rng = np.random.default_rng(100 * geom + len(dt.str))
    chunks = _chunks(dt, shape, 11, rng, nan=True)
    for mi, miss in enumerate(MISSING):
        if miss is not None and dt.kind == "u":
            miss = (7, None, None, 900)
        want = _partials(ctx, st, dt, shape, chunks, axes, miss, shuf, misalign, 0, monkeypatch)
        for cpb in (1, 3, 4, 11, 40):
            got = _partials(ctx, st, dt, shape, chunks, axes, miss, shuf, misalign, cpb, monkeypatch)
            assert got.tobytes() == want.tobytes(), f"{dt} {shape} axes={axes} miss={mi} cpb={cpb}"


@pytest.mark.parametrize("geom", range(len(GEOMS)))
def test_stream_matches_oracle(gpu, monkeypatch, geom):
    """Counts, min/max and sums of the streamed partials against storage.py's
    per-chunk reduction (the sign of a zero extreme is set later, by the tie
    pass, and is checked in test_gpu_zero_sign.py)."""
    from pyactivestorage_amd.device import get_context
    shape, axes = GEOMS[geom]
    dt = np.dtype("<f4")
    ctx = get_context(0)
    st = ctx.thread_stream()
    rng = np.random.default_rng(7 + geom)
    chunks = _chunks(dt, shape, 9, rng, nan=False)
    miss = (-999, None, -50, 140)
    got = _partials(ctx, st, dt, shape, chunks, axes, miss, False, False, 4, monkeypatch)
    sel = tuple(slice(0, n, 1) for n in shape)
    for k, a in enumerate(chunks):
        vals, n = ref.reduce_chunk_bytes(a.tobytes(), None, None, miss, dt, shape, "C", sel, axes, None)
        vm = np.ma.asarray(vals)
        cnt = np.ma.count(vm, axis=axes, keepdims=True).reshape(-1)
        np.testing.assert_array_equal(got[k]["count"], cnt)
        ok = cnt > 0
        for f, fn in (("min", np.ma.min), ("max", np.ma.max)):
            w = np.ma.getdata(fn(vm, axis=axes, keepdims=True)).reshape(-1)[ok]
            np.testing.assert_array_equal(got[k][f][ok].astype(np.float32), w, err_msg=f"chunk {k} {f}")
        wsum = np.ma.filled(vm.astype(np.float64), 0).sum(axis=axes, keepdims=True).reshape(-1)
        np.testing.assert_allclose(got[k]["sum"][ok], wsum[ok], rtol=1e-6, atol=1e-3)


def test_auto_choice_at_size(gpu):
    """The configurations pyas_reduce_axes picks by itself at a C3-like size
    against the one-chunk-per-workgroup kernel and the oracle
    (tests/_axes_stream_auto.py in a fresh process: torch initialises the
    GPU first there; this process already holds libpyas_hip's context)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", "-m", "tests._axes_stream_auto"], cwd=root,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert "axes-stream-auto OK" in r.stdout
    print(r.stdout.strip())
