"""pyas_reduce_axes_grid (chunk layers folded inside the dense column
or LDS row kernel, one launch) against the two-step path it replaces
(pyas_reduce_axes -> per-chunk partial arrays -> pyas_combine_grid), which
follows ``Active._from_storage``'s combine (``activestorage/active.py:
487-516,575-598``).  The combined partials must agree bit for bit: sums,
counts, min/max and NaN propagation, for rounded variable-dtype sums, masked
and unmasked variables, byte-swapped dtypes, several chunk grids and axis
sets, with and without split reduced ranges.  The final results are also
checked against NumPy's masked reductions of the whole array.
"""
import os
import tempfile

import numpy as np
import pytest

from pyactivestorage_amd import active as active_mod
from pyactivestorage_amd import engine
from pyactivestorage_amd.active import Active
from pyactivestorage_amd.variable import ChunkedVariable
from tests._compare import shuffle_bytes

pytestmark = pytest.mark.gpu

FILL = -999


@pytest.fixture(autouse=True)
def _default_floor(gpu):
    yield
    gpu.set_fold_min_blocks(0)


def _variable(shape, chunks, dtype, rng, masked, nan=False, shuffle=False):
    dt = np.dtype(dtype)
    if dt.kind == "f":
        data = rng.uniform(-100, 100, size=shape).astype(dt)
        if nan:
            data.reshape(-1)[rng.choice(data.size, 3, replace=False)] = np.nan
    else:
        data = rng.integers(-50 if dt.kind == "i" else 0, 100, size=shape).astype(dt)
    attrs = {}
    if masked:
        data.reshape(-1)[rng.random(data.size) < 0.2] = FILL if dt.kind != "u" else 7
        attrs["_FillValue"] = np.array([FILL if dt.kind != "u" else 7], dtype=dt)
    path = os.path.join(tempfile.mkdtemp(), "v.chunks")
    index, pos = {}, 0
    with open(path, "wb") as fh:
        for cc in np.ndindex(*[s // c for s, c in zip(shape, chunks)]):
            sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(cc, chunks))
            b = np.ascontiguousarray(data[sl])
            b = shuffle_bytes(b, dt.itemsize) if shuffle else b.tobytes()
            fh.write(b)
            index[cc] = (pos, len(b))
            pos += len(b)
    var = ChunkedVariable(name="v", shape=shape, chunks=chunks, dtype=dt, chunk_index=index,
                          attrs=attrs, filename=path,
                          filter_pipeline=[{"filter_id": 2}] if shuffle else None)
    return var, data


_FIELDS = {"mean": ["sum", "count"], "min": ["min", "count"], "max": ["max", "count"]}


def _same_final(f1, f0, method="mean"):
    """The fields a method reads of the combined partials, byte for byte (the
    two-step path's per-chunk records carry only those: pyas_reduce_axes_ex)."""
    for k in _FIELDS[method]:
        assert f1[k].tobytes() == f0[k].tobytes(), (method, k)


def _partials(var, axis, index, fold, monkeypatch, method="mean"):
    """Combined partials of an Active query (mean by default), raw (before
    formatting)."""
    monkeypatch.setattr(active_mod, "_AXES_FOLD", fold)
    calls = []
    real = engine.reduce_axes_grid

    def spy(*a, **k):
        real(*a, **k)
        calls.append(1)
    monkeypatch.setattr(engine, "reduce_axes_grid", spy)
    a = Active(var, axis=axis)
    a.method = method
    got = {}

    def raw(ctx, st, fin, n, shape):
        final = np.zeros(n, dtype=engine.partial_dtype(var.dtype))
        ctx.d2h(final, fin.ptr, st)
        ctx.synchronize(st)
        got["final"] = final
        return a._format(final.reshape(shape), shape)
    a._format_device = raw
    res = a[index]
    return got["final"], res, len(calls)


CASES = [
    # shape, chunks, axis, index
    ((64, 48, 32), (16, 16, 16), (0,), np.s_[...]),
    ((64, 48, 32), (16, 16, 16), (1,), np.s_[...]),
    ((64, 48, 32), (16, 16, 16), (0, 1), np.s_[...]),
    ((32, 32, 64), (8, 16, 64), (0,), np.s_[8:24, :, :]),
    ((32, 32, 64), (8, 16, 64), (1,), np.s_[:, 16:32, :]),
    ((16, 12, 20, 24), (4, 6, 5, 8), (0, 2), np.s_[...]),
    ((16, 12, 20, 24), (4, 6, 5, 8), (1,), np.s_[4:16]),
    ((128, 8), (32, 8), (0,), np.s_[...]),
    ((20, 256), (5, 256), (0,), np.s_[...]),       # few outputs per chunk: split reduced rows
    ((6, 1024, 8), (3, 128, 8), (0, 1), np.s_[...]),
    # innermost dims reduced, runs <= 256 B: the LDS row layout's fold
    ((32, 32, 32), (8, 16, 32), (2,), np.s_[...]),
    ((16, 12, 40), (4, 6, 20), (2,), np.s_[...]),   # 5 vectors per f4 run: one lane per output
    ((16, 12, 20, 24), (4, 6, 5, 8), (3,), np.s_[4:16]),
    ((24, 96), (8, 32), (1,), np.s_[...]),
    ((40, 8, 32), (8, 8, 32), (2,), np.s_[...]),   # 64 outputs per chunk: a partial last tile
    # >= 256 items per chunk, no split, rows a multiple of 4: the lean column fold
    ((32, 64, 64), (8, 16, 64), (0,), np.s_[...]),
    ((8, 64, 256), (8, 16, 256), (1,), np.s_[...]),
    ((36, 32, 96), (12, 16, 96), (0,), np.s_[12:36]),
    ((30, 32, 64), (10, 16, 64), (0,), np.s_[...]),   # 10 rows: not whole 4-row groups, k_axes_fold
]
LEAN_CASES = (15, 16, 17)


@pytest.mark.parametrize("dtype", ["<f4", ">f4", "<f8", "<i4", "<u4", "<i8"])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_fold_matches_two_step(gpu, dtype, masked, case, monkeypatch):
    gpu.set_fold_min_blocks(1)            # small test grids: fold whatever the size
    shape, chunks, axis, index = CASES[case]
    rng = np.random.default_rng(case * 31 + len(dtype))
    var, data = _variable(shape, chunks, dtype, rng, masked, nan=(case in (0, 15)))
    f1, r1, n1 = _partials(var, axis, index, True, monkeypatch)
    f0, r0, n0 = _partials(var, axis, index, False, monkeypatch)
    assert n1 == 1 and n0 == 0            # the fold ran, then the two-step path
    _same_final(f1, f0)
    for method in ("min", "max"):         # the two-step path's min / max records
        g1, _, _ = _partials(var, axis, index, True, monkeypatch, method)
        g0, _, _ = _partials(var, axis, index, False, monkeypatch, method)
        _same_final(g1, g0, method)
    # and the result against NumPy's masked mean of the selection
    sel = data[index]
    m = np.ma.masked_equal(sel, var.attrs["_FillValue"][0]) if masked else np.ma.MaskedArray(sel)
    want = np.ma.mean(m.astype(np.float64), axis=axis, keepdims=True)
    want = np.ma.masked_invalid(want)     # np.ma's out / n (active.py:630) masks NaN means
    np.testing.assert_array_equal(np.ma.getmaskarray(r1), np.ma.getmaskarray(want))
    ok = ~np.ma.getmaskarray(want)
    np.testing.assert_allclose(np.ma.getdata(r1)[ok], np.ma.getdata(want)[ok], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("dtype", ["<f4", ">f8", "<i4"])
@pytest.mark.parametrize("case", [0, 1, 2, 5, 8, 10, 11, 14, 16])
def test_fold_shuffled_matches_two_step(gpu, dtype, case, monkeypatch):
    """Byte-shuffled chunks (the un-shuffle fused into the dense loads, one
    piece per byte plane): fold == two-step bit for bit, and the same result
    as the unshuffled variable (same summation order, so bit-identical)."""
    gpu.set_fold_min_blocks(1)
    shape, chunks, axis, index = CASES[case]
    rng = np.random.default_rng(case * 7 + len(dtype))
    var, data = _variable(shape, chunks, dtype, rng, True, nan=(case in (0, 16)), shuffle=True)
    f1, r1, n1 = _partials(var, axis, index, True, monkeypatch)
    f0, r0, n0 = _partials(var, axis, index, False, monkeypatch)
    # case 11's 20-element runs are not whole 16-element shuffled load units:
    # the fold refuses and the two-step (generic kernel) path runs
    assert n1 == (0 if case == 11 else 1) and n0 == 0
    _same_final(f1, f0)
    rng = np.random.default_rng(case * 7 + len(dtype))
    plain, _ = _variable(shape, chunks, dtype, rng, True, nan=(case in (0, 16)), shuffle=False)
    fp, rp, _ = _partials(plain, axis, index, True, monkeypatch)
    if case != 11:     # same kernel, same order: bit-identical
        assert fp.tobytes() == f1.tobytes()
    else:              # generic kernel vs dense fold: sums differ only in order
        # (the two-step path keeps sum + count records for mean queries)
        np.testing.assert_array_equal(fp["count"], f1["count"])
        for method in ("min", "max"):
            g_p, _, _ = _partials(plain, axis, index, True, monkeypatch, method)
            g_s, _, _ = _partials(var, axis, index, True, monkeypatch, method)
            _same_final(g_p, g_s, method)
        # chunk sums are rounded to f32 (active.py:512) and these data cancel
        np.testing.assert_allclose(fp["sum"], f1["sum"], rtol=1e-6, atol=1e-3)


def test_fold_refuses_long_rows(gpu, monkeypatch):
    """Innermost dim reduced with 512-B runs: neither the column nor the LDS
    row layout, so the two-step path runs."""
    gpu.set_fold_min_blocks(1)
    rng = np.random.default_rng(3)
    var, data = _variable((32, 32, 128), (8, 16, 128), "<f4", rng, True)
    f, r, n = _partials(var, (2,), np.s_[...], True, monkeypatch)
    assert n == 0
    f0, r0, _ = _partials(var, (2,), np.s_[...], False, monkeypatch)
    _same_final(f, f0)


def test_fold_refuses_too_few_workgroups(gpu, monkeypatch):
    """Few kept-dim columns and many layers: the fold would launch too few
    workgroups, so the two-step path runs (same result)."""
    gpu.set_fold_min_blocks(0)            # the default floor (2048)
    rng = np.random.default_rng(4)
    var, data = _variable((64, 48, 32), (16, 16, 16), "<f4", rng, True)
    f, r, n = _partials(var, (0, 1), np.s_[...], True, monkeypatch)
    assert n == 0
    gpu.set_fold_min_blocks(1)
    f1, r1, n1 = _partials(var, (0, 1), np.s_[...], True, monkeypatch)
    assert n1 == 1
    _same_final(f1, f)
    gpu.set_fold_min_blocks(0)


@pytest.mark.parametrize("lean", ["1", "2"])
@pytest.mark.parametrize("dtype", ["<f4", "<f8", "<i4"])
@pytest.mark.parametrize("case", LEAN_CASES)
def test_lean_fold_matches_split_fold(gpu, dtype, case, lean, monkeypatch):
    """k_axes_fold_lean (PYAS_FOLD_LEAN=1: one lane per column item; 2: the
    column's layers split over two lanes, the second half's per-layer sums
    handed over in LDS) against k_axes_fold (PYAS_FOLD_LEAN=0) and the
    two-step path, bit for bit, on data with signed zeros in every layer and
    NaN: the lean kernel folds layer min/max straight into the running
    min/max with merge's pmin/pmax, which must keep the same zero sign."""
    gpu.set_fold_min_blocks(1)
    monkeypatch.setenv("PYAS_FOLD_LEAN", lean)
    shape, chunks, axis, index = CASES[case]
    rng = np.random.default_rng(case * 13 + len(dtype))
    var, data = _variable(shape, chunks, dtype, rng, True, nan=True)
    if np.dtype(dtype).kind == "f":
        flat = data.reshape(-1)
        z = rng.choice(flat.size, flat.size // 5, replace=False)
        flat[z] = np.where(rng.random(z.size) < 0.5, -0.0, 0.0).astype(data.dtype)
        flat[rng.choice(flat.size, 2, replace=False)] = np.nan
        var, data = _rewrite(var, data)
    f_lean, r_lean, n_lean = _partials(var, axis, index, True, monkeypatch)
    monkeypatch.setenv("PYAS_FOLD_LEAN", "0")
    f_split, _, n_split = _partials(var, axis, index, True, monkeypatch)
    f_two, _, n_two = _partials(var, axis, index, False, monkeypatch)
    assert n_lean == 1 and n_split == 1 and n_two == 0
    assert f_lean.tobytes() == f_split.tobytes()
    _same_final(f_lean, f_two)
    for method in ("min", "max"):         # the two-step path's min / max records
        monkeypatch.setenv("PYAS_FOLD_LEAN", lean)
        g_lean, _, _ = _partials(var, axis, index, True, monkeypatch, method)
        g_two, _, _ = _partials(var, axis, index, False, monkeypatch, method)
        _same_final(g_lean, g_two, method)


def _rewrite(var, data):
    """Write `data` back into var's chunk file (same layout, unshuffled)."""
    with open(var.filename, "r+b") as fh:
        for cc, (pos, n) in var.chunk_index.items():
            sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(cc, var.chunks))
            fh.seek(pos)
            fh.write(np.ascontiguousarray(data[sl]).tobytes())
    return var, data


WAVE_CASES = [
    # many chunk layers per output: pyas_combine_grid's one-wave-per-output form
    ((130, 8, 16), (1, 4, 16), (0,), np.s_[...]),                   # 130 layers: 2 full tiles + 2
    ((10, 12, 64), (1, 1, 64), (0, 1), np.s_[...]),                 # 120 layers
    ((3, 40, 8, 24), (1, 1, 4, 8), (0, 1), np.s_[:, 3:37, 1:7, 5:20]),   # 102 layers, hyperslab tables
    ((4, 96, 8), (2, 1, 8), (1,), np.s_[1:4, :, 2:8]),              # 96 layers between kept dims
    ((64, 4, 8), (2, 4, 8), (0,), np.s_[...]),                      # 32 layers: the threshold
]


@pytest.mark.parametrize("dtype", ["<f4", ">f4", "<f8", "<i4"])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("case", range(len(WAVE_CASES)))
def test_combine_grid_wave_matches_thread(gpu, dtype, masked, case, monkeypatch):
    """k_combine_grid_wave (one wave per output; lanes load 64 layers into
    LDS, lane 0 merges them in layer order) against k_combine_grid
    (PYAS_COMBINE_WAVE=0, one thread per output), bit for bit, on the
    two-step path, with signed zeros and NaN in the data; then the result
    against NumPy's masked mean of the selection."""
    shape, chunks, axis, index = WAVE_CASES[case]
    rng = np.random.default_rng(case * 17 + len(dtype) + masked)
    var, data = _variable(shape, chunks, dtype, rng, masked, nan=True)
    if np.dtype(dtype).kind == "f":
        flat = data.reshape(-1)
        z = rng.choice(flat.size, flat.size // 5, replace=False)
        flat[z] = np.where(rng.random(z.size) < 0.5, -0.0, 0.0).astype(data.dtype)
        var, data = _rewrite(var, data)
    monkeypatch.delenv("PYAS_COMBINE_WAVE", raising=False)
    f_wave, r_wave, n_wave = _partials(var, axis, index, False, monkeypatch)
    monkeypatch.setenv("PYAS_COMBINE_WAVE", "0")
    f_thr, _, n_thr = _partials(var, axis, index, False, monkeypatch)
    assert n_wave == 0 and n_thr == 0       # the two-step path both times
    assert f_wave.tobytes() == f_thr.tobytes()
    sel = data[index]
    m = (np.ma.masked_equal(sel, var.attrs["_FillValue"][0]) if masked else np.ma.MaskedArray(sel))
    want = np.ma.masked_invalid(np.ma.mean(m.astype(np.float64), axis=axis, keepdims=True))
    np.testing.assert_array_equal(np.ma.getmaskarray(r_wave), np.ma.getmaskarray(want))
    ok = ~np.ma.getmaskarray(want)
    np.testing.assert_allclose(np.ma.getdata(r_wave)[ok], np.ma.getdata(want)[ok], rtol=1e-5, atol=1e-4)
