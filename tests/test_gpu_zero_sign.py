"""NumPy's sign of a zero min/max on the device (pyas_tie_chunks /
pyas_tie_grid / pyas_tie_segments / pyas_tie_finalize; the rule and its
host restatement are in zerosign.py, checked against NumPy by
tests/test_zero_sign.py).

Per chunk (``storage.py:95-100``): the drop-in returns the reference's +0.0
/ -0.0 for every axis subset and selection: masked chunks (``np.ma`` reduces
a filled copy), unmasked strided and reversed views (NumPy reduces the view
itself), index lists (a copy laid out with the listed dim outermost),
big-endian and F-ordered chunks.  Across chunks (``active.py:575-598``):
``Active`` stores the per-chunk results in the ``out`` array and reduces it
with ``np.ma.min/max`` again, here restated with the oracle's own
``reduce_chunk`` and ``combine_partials`` for full and partial-axis queries,
resident or not, folded in the kernel or in two steps, and under a group of
ranks (gloo, sharing this GPU).  Every comparison is of bytes: a zero's
sign bit included.
"""
import threading

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import active as active_mod
from pyactivestorage_amd import storage as pas
from pyactivestorage_amd.active import Active
from pyactivestorage_amd.variable import ChunkedVariable
from pyactivestorage_amd.zerosign import tie_rule

pytestmark = pytest.mark.gpu


def _same_bytes(want, got, what):
    w = np.asarray(np.ma.getdata(want))
    g = np.asarray(np.ma.getdata(got))
    assert w.shape == g.shape and w.dtype == g.dtype, (what, w.shape, g.shape, w.dtype, g.dtype)
    assert np.array_equal(np.ma.getmaskarray(want), np.ma.getmaskarray(got)), what
    keep = ~np.ma.getmaskarray(want)
    wk, gk = w[keep], g[keep]
    nan = np.isnan(wk)
    assert np.array_equal(nan, np.isnan(gk)), what
    assert wk[~nan].tobytes() == gk[~nan].tobytes(), (what, wk[~nan][wk[~nan] != gk[~nan]],
                                                     np.signbit(wk[~nan]).sum(), np.signbit(gk[~nan]).sum())


def _chunk(rng, shape, dt, pattern, dens=0.3, n_fill=10):
    n = int(np.prod(shape))
    if pattern == "zeros":
        a = np.zeros(n, dtype=dt)
    else:
        a = rng.uniform(0.5, 9.0, n).astype(dt) * (1 if pattern == "min0" else -1)
    z = rng.random(n) < dens
    a[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
    a[rng.choice(n, n_fill, replace=False)] = -999.0
    return a.reshape(shape)


SELS = [(slice(None),) * 3, (slice(1, 11), slice(2, 19), slice(0, 66, 3)),
        (slice(11, 0, -2), slice(None), slice(60, 3, -1)), (slice(None), [0, 3, 4, 17], slice(5, 50)),
        (2, slice(None), slice(None, None, 4))]
AXES = [(0,), (1,), (2,), (0, 1), (1, 2), (0, 2), (0, 1, 2)]


@pytest.mark.parametrize("dt", ["<f4", ">f8"])
@pytest.mark.parametrize("pattern", ["min0", "max0", "zeros"])
@pytest.mark.parametrize("order", ["C", "F"])
@pytest.mark.parametrize("group", ["", "1", "16", "64"])
def test_per_call_chunk_sign(gpu, dt, pattern, order, group, monkeypatch):
    """storage.py:95-100 per call: every selection kind x axis subset, with
    and without a mask attribute, against the oracle byte for byte.  The
    level-1 backward scan (k_tie_scan) runs with the host's choice of lanes
    per output ("") and forced to each layout (PYAS_TIE_GROUP): the result
    may not depend on it."""
    monkeypatch.setenv("PYAS_TIE_GROUP", group)
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(len(dt) * 7 + len(pattern) + len(order))
    shape = (12, 20, 70)                               # > one 8192-element iterator piece
    a = _chunk(rng, shape, np.dtype(dt), pattern)
    raw = (np.asfortranarray(a) if order == "F" else a).tobytes(order="A")
    methods = (np.ma.min, np.min) if pattern != "max0" else (np.ma.max, np.max)
    for miss in ((None, None, None, None), (np.dtype(dt).type(-999.0), None, None, None)):
        for sel in SELS:
            for axis in AXES:
                if isinstance(sel[0], int):   # dim 0 dropped: a 2-D result
                    axis = tuple(sorted({min(x, 1) for x in axis}))
                for method in methods:
                    want, wn = ref.reduce_chunk_bytes(raw, None, None, miss, dt, shape, order, sel, axis, method)
                    got, gn = pas.reduce_chunk_bytes(raw, None, None, miss, dt, shape, order, sel, axis, method)
                    _same_bytes(want, got, (miss[0], sel, axis, method.__name__))
                    assert np.array_equal(wn, gn)


def _variable(a, chunks, attrs):
    shape = a.shape
    grid = [-(-s // c) for s, c in zip(shape, chunks)]
    blobs, index, pos = [], {}, 0
    for cc in np.ndindex(*grid):
        blk = np.full(chunks, -999.0, dtype=a.dtype)   # edge chunks padded like HDF5
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(cc, chunks, shape))
        blk[tuple(slice(0, x.stop - x.start) for x in sl)] = a[sl]
        b = blk.tobytes()
        index[cc] = (pos, len(b))
        blobs.append(b)
        pos += len(b)
    data = b"".join(blobs)
    return ChunkedVariable(name="v", shape=shape, chunks=chunks, dtype=a.dtype.str, chunk_index=index,
                           attrs=attrs, reader=lambda off, size: data[off:off + size]), data


def _reference_active(a, chunks, index, axis, kind, missing, data_of):
    """active.py:487-630 over storage.py's reduce_chunk (the oracle's),
    for an index of positive-step slices."""
    shape = a.shape
    picks, per_dim = [], []
    for d, s in enumerate(index):
        idx = np.arange(shape[d])[s]
        c = chunks[d]
        coords = sorted(set((idx // c).tolist()))
        per_dim.append([(k, idx[idx // c == k]) for k in coords])
    out_shape = [len(per_dim[d]) if d in axis else sum(len(x) for _, x in per_dim[d]) for d in range(a.ndim)]
    method = np.ma.min if kind == "min" else np.ma.max
    parts = []
    for combo in np.ndindex(*[len(p) for p in per_dim]):
        cc, csel, osel = [], [], []
        for d, j in enumerate(combo):
            k, ids = per_dim[d][j]
            cc.append(k)
            step = index[d].step or 1
            local = ids - k * chunks[d]
            csel.append(slice(int(local[0]), int(local[-1]) + 1, step))
            if d in axis:
                osel.append(slice(j, j + 1))
            else:
                before = sum(len(x) for _, x in per_dim[d][:j])
                osel.append(slice(before, before + len(ids)))
        raw = data_of(tuple(cc))
        tmp, n = ref.reduce_chunk_bytes(raw, None, None, missing, a.dtype.str, chunks, "C", tuple(csel),
                                        tuple(axis), method)
        parts.append((tmp, n, tuple(osel)))
    return ref.combine_partials(parts, out_shape, a.dtype, tuple(axis), kind)


QUERIES = [(slice(None),) * 3, (slice(1, 15), slice(3, 21), slice(2, 75)), (slice(0, 16, 3), slice(None), slice(7, 80, 2))]


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("kind", ["min", "max"])
@pytest.mark.parametrize("fill", [True, False])
@pytest.mark.parametrize("group", ["", "1", "64"])
def test_active_sign(gpu, dt, kind, fill, group, monkeypatch):
    """Active full and partial-axis min/max (fold and two-step paths,
    resident and not) against active.py's combine over storage.py's
    per-chunk results: the zero's sign bit included (level-1 scan layout
    forced by PYAS_TIE_GROUP, or the host's choice)."""
    monkeypatch.setenv("PYAS_TIE_GROUP", group)
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(3 + len(kind) + fill + len(dt))
    shape, chunks = (16, 24, 80), (4, 8, 20)
    a = _chunk(rng, shape, np.dtype(dt), "min0" if kind == "min" else "max0", dens=0.2, n_fill=10 if fill else 0)
    attrs = {"_FillValue": np.array([-999.0], dtype=dt)} if fill else {}
    missing = (np.dtype(dt).type(-999.0), None, None, None) if fill else (None, None, None, None)
    var, data = _variable(a, chunks, attrs)
    data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
    for q in QUERIES:
        for axis in [(0, 1, 2)] + AXES[:6]:
            want = _reference_active(a, chunks, q, axis, kind, missing, data_of)
            for resident in (False, True):
                for fold in (True, False):
                    old = active_mod._AXES_FOLD
                    active_mod._AXES_FOLD = fold
                    try:
                        act = Active(var, axis=axis, resident=resident)
                        act.method = kind
                        got = act[q]
                        act.method = kind                    # (reset after each query, active.py:633)
                        got2 = act[q] if resident else got   # a cached replay
                    finally:
                        active_mod._AXES_FOLD = old
                    _same_bytes(want, got, (q, axis, resident, fold))
                    _same_bytes(want, got2, (q, axis, "replay"))
            active_mod.release_resident(var)


def test_replay_threads_share_a_query(gpu):
    """8 threads replaying ONE cached resident min query on data
    with mixed signed zeros all get the reference's sign (the replay holds
    the query's lock across its launches and copies)."""
    rng = np.random.default_rng(77)
    shape, chunks = (16, 24, 80), (4, 8, 20)
    a = _chunk(rng, shape, np.dtype("<f4"), "min0", dens=0.1)
    var, data = _variable(a, chunks, {"_FillValue": np.array([-999.0], dtype="<f4")})
    data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
    missing = (np.float32(-999.0), None, None, None)
    for axis in ((0, 1, 2), (0,), (0, 2)):
        want = _reference_active(a, chunks, (slice(None),) * 3, axis, "min", missing, data_of)
        act = Active(var, axis=axis, resident=True)
        act.method = "min"
        act[...]
        errors = []

        def worker():
            try:
                for _ in range(20):
                    x = Active(var, axis=axis, resident=True)
                    x.method = "min"
                    _same_bytes(want, x[...], axis)
            except Exception as exc:   # noqa: BLE001 - reported below
                errors.append(exc)
        ts = [threading.Thread(target=worker) for _ in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors[0]
    active_mod.release_resident(var)


@pytest.mark.parametrize("group", ["", "1", "16"])
def test_strided_full_reduction_sign(gpu, group, monkeypatch):
    """a full reduction of an unmasked strided view whose
    kept block is empty (a 1-D chunk[::k], or (8,12,40)[2:5,:,::4] reduced
    over every dim) is one strided call per run (NumPy's acc loop), not a
    copied contiguous call.  Dense signed zeros, compared byte for byte with
    NumPy through the oracle."""
    monkeypatch.setenv("PYAS_TIE_GROUP", group)
    if tie_rule("<f4") is None or tie_rule("<f8") is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(590)
    none = (None, None, None, None)
    n_cases = 0
    for dt in ("<f4", "<f8"):
        for n in (7, 64, 300, 4100, 20000):
            for step in (2, 3, 5, -2, 16):
                for dens in (0.3, 0.9):
                    a = rng.uniform(0.5, 9.0, n).astype(dt)
                    z = rng.random(n) < dens
                    a[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
                    inner = slice(1, n - 1, step) if step > 0 else slice(n - 2, 0, step)
                    for sel in ((slice(None, None, step),), (inner,)):
                        for method in (np.ma.min, np.min):
                            want, wn = ref.reduce_chunk_bytes(a.tobytes(), None, None, none, dt, (n,), "C", sel,
                                                              (0,), method)
                            got, gn = pas.reduce_chunk_bytes(a.tobytes(), None, None, none, dt, (n,), "C", sel,
                                                             (0,), method)
                            _same_bytes(want, got, (dt, n, sel, method.__name__))
                            assert np.array_equal(wn, gn)
                            n_cases += 1
        shape = (8, 12, 40)
        for rep in range(24):
            a = rng.uniform(0.5, 9.0, shape).astype(dt)
            z = rng.random(shape) < 0.6
            a[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
            for sel in ((slice(2, 5), slice(None), slice(None, None, 4)),
                        (slice(None), slice(3, 9), slice(1, None, 3)),
                        (slice(None, None, 2), slice(None), slice(None, None, 8))):
                for axis in ((0, 1, 2), (1, 2), (0, 2)):
                    want, _ = ref.reduce_chunk_bytes(a.tobytes(), None, None, none, dt, shape, "C", sel, axis,
                                                     np.min)
                    got, _ = pas.reduce_chunk_bytes(a.tobytes(), None, None, none, dt, shape, "C", sel, axis,
                                                    np.min)
                    _same_bytes(want, got, (dt, rep, sel, axis))
                    n_cases += 1
    assert n_cases >= 800


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("lean", ["1", "2"])
@pytest.mark.parametrize("kind", ["min", "max"])
def test_fused_fold_sign(gpu, dt, lean, kind, monkeypatch):
    """PYAS_FOLD_ZERO_SIGN_*: where both NumPy reductions are elementwise
    (innermost dim kept, C order), the lean column fold tracks the last zero
    itself.  Its bytes must equal the zero-sign passes' (the same query with
    the fusion refused) and active.py's combine over storage.py's results,
    for the unsplit and the layer-split lean kernel."""
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    monkeypatch.setenv("PYAS_FOLD_LEAN", lean)
    gpu.set_fold_min_blocks(1)
    try:
        rng = np.random.default_rng(17 + len(lean) + len(kind))
        shape, chunks = (32, 32, 128), (16, 16, 64)
        a = _chunk(rng, shape, np.dtype(dt), "min0" if kind == "min" else "max0", dens=0.4, n_fill=40)
        attrs = {"_FillValue": np.array([-999.0], dtype=dt)}
        missing = (np.dtype(dt).type(-999.0), None, None, None)
        var, data = _variable(a, chunks, attrs)
        data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
        calls = []
        real = active_mod.Active._fold

        def spy(self, *args):
            fused = real(self, *args)
            calls.append(fused)
            return fused
        monkeypatch.setattr(active_mod.Active, "_fold", spy)
        for axis in ((0,), (1,)):
            want = _reference_active(a, chunks, (slice(None),) * 3, axis, kind, missing, data_of)
            for resident in (False, True):
                act = Active(var, axis=axis, resident=resident)
                act.method = kind
                got = act[...]
                _same_bytes(want, got, (axis, resident, "fused"))
                if resident:   # the cached replay folds with the fusion again
                    act.method = kind
                    _same_bytes(want, act[...], (axis, "replay"))
            active_mod.release_resident(var)
        assert calls and all(calls), calls   # the lean kernel took every query with the fusion
        monkeypatch.setattr(active_mod.Active, "_fold_sign_ok", lambda self, axes: False)
        for axis in ((0,), (1,)):
            want = _reference_active(a, chunks, (slice(None),) * 3, axis, kind, missing, data_of)
            act = Active(var, axis=axis)
            act.method = kind
            _same_bytes(want, act[...], (axis, "passes"))
    finally:
        gpu.set_fold_min_blocks(0)


ROW_FOLD_CASES = [   # (shape, chunks, axis): each output row of a chunk one contiguous NumPy call
    ((32, 64, 128), (16, 32, 32), (2,)),     # the innermost dim; `out` call over 4 layers
    ((32, 64, 128), (16, 4, 8), (1, 2)),     # a two-dim trailing group (32); `out` call of 16 x 16
    ((32, 64, 128), (1, 16, 32), (0, 2)),    # extent-1 reduced dim; `out`: 32 runs of 4 layers
    ((32, 32, 4), (16, 16, 1), (1,)),        # extent-1 kept innermost dim: `out` elementwise
]


@pytest.mark.parametrize("dt", ["<f4", ">f4", "<f8"])
@pytest.mark.parametrize("row_lds", ["1", "2", "4"])
@pytest.mark.parametrize("dens", [0.4, 0.03])
@pytest.mark.parametrize("kind", ["min", "max"])
@pytest.mark.parametrize("case", range(len(ROW_FOLD_CASES)))
def test_fused_row_fold_sign(gpu, dt, row_lds, dens, kind, case, monkeypatch):
    """PYAS_FOLD_ZERO_SIGN_* in the LDS row fold (k_axes_fold_row, 1, 2 or 4
    lanes per row): each row whose min/max is a zero is keyed by the host's
    NumPy rule from the tile in LDS, and its sign at its layer's position in
    the `out` array's call.  Bytes equal active.py's combine over
    storage.py's results and the zero-sign passes' (the fusion refused)."""
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    monkeypatch.setenv("PYAS_ROW_LDS", row_lds)
    gpu.set_fold_min_blocks(1)
    try:
        shape, chunks, axis = ROW_FOLD_CASES[case]
        rng = np.random.default_rng(case * 31 + len(dt) + int(row_lds) + int(dens * 100) + len(kind))
        a = _chunk(rng, shape, np.dtype(dt), "min0" if kind == "min" else "max0", dens=dens, n_fill=60)
        attrs = {"_FillValue": np.array([-999.0], dtype=dt)}
        missing = (np.dtype(dt).type(-999.0), None, None, None)
        var, data = _variable(a, chunks, attrs)
        data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
        calls = []
        real = active_mod.Active._fold

        def spy(self, *args):
            fused = real(self, *args)
            calls.append(fused)
            return fused
        monkeypatch.setattr(active_mod.Active, "_fold", spy)
        want = _reference_active(a, chunks, (slice(None),) * 3, axis, kind, missing, data_of)
        for resident in (False, True):
            act = Active(var, axis=axis, resident=resident)
            act.method = kind
            _same_bytes(want, act[...], (axis, resident, "fused"))
            if resident:   # the cached replay folds with the fusion again
                act.method = kind
                _same_bytes(want, act[...], (axis, "replay"))
        active_mod.release_resident(var)
        assert calls and all(calls), calls   # the row kernel took the fusion every time
        monkeypatch.setattr(active_mod.Active, "_fold_sign_ok", lambda self, axes: False)
        act = Active(var, axis=axis)
        act.method = kind
        _same_bytes(want, act[...], (axis, "passes"))
    finally:
        gpu.set_fold_min_blocks(0)


@pytest.mark.parametrize("dt", ["<f4", ">f4", "<f8"])
@pytest.mark.parametrize("dens", [0.5, 0.02, 0.0005])
@pytest.mark.parametrize("kind", ["min", "max"])
def test_full_reduction_pick(gpu, dt, dens, kind):
    """pyas_tie_chunks_total: Active full min/max scans only the two chunks
    the level-2 keys can pick (K1's and W's, by position alone).  Dense,
    sparse and very sparse zeros over 256 chunks, against active.py's
    combine over storage.py's per-chunk results, sign bit included."""
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(int(dens * 10000) + len(dt) + len(kind))
    shape, chunks = (64, 64, 64), (16, 8, 8)
    a = _chunk(rng, shape, np.dtype(dt), "min0" if kind == "min" else "max0", dens=dens, n_fill=30)
    attrs = {"_FillValue": np.array([-999.0], dtype=dt)}
    missing = (np.dtype(dt).type(-999.0), None, None, None)
    var, data = _variable(a, chunks, attrs)
    data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
    for q in QUERIES[:2]:
        want = _reference_active(a, chunks, q, (0, 1, 2), kind, missing, data_of)
        for resident in (False, True):
            act = Active(var, resident=resident)
            act.method = kind
            _same_bytes(want, act[q], (q, resident))
        active_mod.release_resident(var)


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("kind", ["min", "max"])
@pytest.mark.parametrize("dens", [0.5, 0.02])
def test_walk_keyed_level1_sign(gpu, dt, kind, dens):
    """The two-step path over a hyperslab whose edge chunks are cut boxes:
    the column walk keys level 1 of NumPy's zero sign itself
    (PYAS_REC_ZERO_SIGN, the last zero in row order wins) instead of
    pyas_tie_chunks; dense and sparse zeros, min and max, against the
    reference's combine over storage.py's results (sign bit included).  The
    fused path must actually run for the column-layout axis sets, and with
    the `out` calls elementwise pyas_combine_grid keys level 2 (the last zero
    layer wins, PYAS_FOLD_ZERO_SIGN_*) so no tie pass runs.  The replay goes
    through _CachedQuery's same two launches."""
    if tie_rule(dt) is None:
        pytest.skip("no NumPy tie rule derived on this host")
    rng = np.random.default_rng(41 + int(dens * 100) + len(kind))
    shape, chunks = (32, 48, 64), (16, 16, 32)
    a = _chunk(rng, shape, np.dtype(dt), "min0" if kind == "min" else "max0", dens=dens, n_fill=10)
    attrs = {"_FillValue": np.array([-999.0], dtype=dt)}
    missing = (np.dtype(dt).type(-999.0), None, None, None)
    var, data = _variable(a, chunks, attrs)
    data_of = lambda cc: data[var.chunk_index[cc][0]: var.chunk_index[cc][0] + var.chunk_index[cc][1]]
    q = (slice(1, 31), slice(1, 47), slice(1, 63))
    old = active_mod._AXES_FOLD
    active_mod._AXES_FOLD = False
    try:
        for axis in [(0,), (1,), (0, 1), (2,), (1, 2)]:
            want = _reference_active(a, chunks, q, axis, kind, missing, data_of)
            act = Active(var, axis=axis, resident=True)
            act.method = kind
            got = act[q]
            _same_bytes(want, got, (q, axis))
            act.method = kind
            _same_bytes(want, act[q], (q, axis, "replay"))
            plans = list(var._pyas_resident.get("plans", {}).values())
            if 2 not in axis:   # innermost dim kept: the walk keyed level 1, the combine level 2
                assert any(p.grid is not None and p.grid.get("zs1") for p in plans), axis
                assert any(p.grid is not None and p.grid.get("zs2") for p in plans), axis
            elif axis == (2,):   # LDS rows: each row one call, keyed by the walk
                assert any(p.grid is not None and p.grid.get("zs1") for p in plans), axis
            active_mod.release_resident(var)
    finally:
        active_mod._AXES_FOLD = old
