"""``k_axes_shuf_slab``: shuffled chunks whose reduced rows lie inside each
kept-outer block (dense form RO == 1, e.g. axis (1,) of a 64^3 chunk), staged
block by block through LDS.  Its partials must equal the per-chunk column
walk's (``dense_col``, ``PYAS_SHUF_SLAB=0 PYAS_COL_STREAM=0``) byte for byte:
the same 4-row groups in the same order (``storage.py:95-104`` per chunk,
before ``active.py:575-598`` folds them).  Covers 64 and 128 output columns,
several tiles per block (RB < RI), f32/f64/i16 and big-endian data, every
mask mode, NaN, chunk counts that leave waves idle, misaligned chunk
offsets, and the compact records.
"""
import numpy as np
import pytest

from pyactivestorage_amd import _lib
from tests._compare import assert_partials_match_oracle, oracle_partials
from tests.test_gpu_axes_stream import _chunks, _partials

pytestmark = pytest.mark.gpu

# >= 256 column items per chunk (the column layout's split 1, which the
# slab kernel requires): KO * KI / (16 / itemsize) >= 256
GEOMS = [((16, 64, 64), (1,)), ((32, 16, 64), (1,)), ((8, 128, 128), (1,)), ((8, 12, 128), (1,)),
         ((24, 32, 64), (1,)), ((4, 4, 64, 64), (2,))]
DTYPES = ["<f4", ">f4", "<f8", "<i2"]
MISSING = [None, (-999, None, -50, 140), (None, None, -1e30, None), (-999, 77, None, None)]


@pytest.mark.parametrize("misalign", [False, True])
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("geom", range(len(GEOMS)))
def test_slab_equals_column_walk(gpu, monkeypatch, geom, dt, misalign):
    from pyactivestorage_amd.device import get_context
    shape, axes = GEOMS[geom]
    dt = np.dtype(dt)
    ctx = get_context(0)
    st = ctx.thread_stream()
    rng = np.random.default_rng(300 + 10 * geom + len(dt.str))
    n = 5 if geom % 2 else 9
    chunks = _chunks(dt, shape, n, rng, nan=True)
    for mi, miss in enumerate(MISSING):
        if miss is not None and dt.kind == "i":
            miss = (7, None, -500, 900) if mi == 1 else None
        monkeypatch.setenv("PYAS_SHUF_SLAB", "0")
        want = _partials(ctx, st, dt, shape, chunks, axes, miss, True, misalign, 0, monkeypatch)
        monkeypatch.setenv("PYAS_SHUF_SLAB", "1")
        got = _partials(ctx, st, dt, shape, chunks, axes, miss, True, misalign, "", monkeypatch)
        assert got.tobytes() == want.tobytes(), f"{dt} {shape} axes={axes} miss={mi} misalign={misalign}"
        # and straight against the oracle, two chunks per case
        full = tuple(slice(0, m) for m in shape)
        for k in (0, 1):
            assert_partials_match_oracle(got[k], oracle_partials(chunks[k], full, axes, miss), dt,
                                         f"{dt} {shape} axes={axes} miss={mi} chunk {k}")


@pytest.mark.parametrize("method", ["min", "max", "mean"])
def test_active_reaches_slab(gpu, monkeypatch, tmp_path, method):
    """An ``Active`` query that runs ``k_axes_shuf_slab`` end to end (a
    byte-shuffled variable in 64^3 chunks, axis (1,), the two-step path:
    PYAS_AXES_FOLD off), against NumPy over the whole masked variable
    (storage.py:95-104 per chunk, active.py:575-598 across chunks)."""
    from pyactivestorage_amd import active as act_mod
    from pyactivestorage_amd.active import Active
    from pyactivestorage_amd.variable import ChunkedVariable
    from tests._compare import shuffle_bytes
    monkeypatch.setattr(act_mod, "_AXES_FOLD", False)
    rng = np.random.default_rng(77)
    shape, chunks = (64, 128, 64), (64, 64, 64)
    data = rng.uniform(1, 1000, size=shape).astype("<f4")
    data.reshape(-1)[rng.random(data.size) < 0.03] = -999.0
    path = tmp_path / "shuf.chunks"
    index = {}
    with open(path, "wb") as f:
        off = 0
        for j in range(2):
            raw = shuffle_bytes(np.ascontiguousarray(data[:, 64 * j:64 * (j + 1), :]), 4)
            f.write(raw)
            index[(0, j, 0)] = (off, len(raw))
            off += len(raw)
    var = ChunkedVariable(name="s", shape=shape, chunks=chunks, dtype=np.dtype("<f4"), chunk_index=index,
                          attrs={"_FillValue": np.array([-999.0], dtype="<f4")}, filename=str(path),
                          filter_pipeline=[{"filter_id": 2, "client_data": [4]}])
    a = Active(var)
    getattr(a, method)(axis=(1,))
    got = a[...]
    m = np.ma.masked_equal(data, np.float32(-999.0))
    want = getattr(np.ma, method)(m, axis=1, keepdims=True)
    assert got.shape == want.shape
    if method == "mean":
        np.testing.assert_allclose(np.ma.getdata(got), np.ma.getdata(want), rtol=1e-6)
    else:
        assert np.ma.getdata(got).tobytes() == np.ma.getdata(want).astype("<f4").tobytes()
