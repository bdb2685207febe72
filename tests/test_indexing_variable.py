"""CPU tests: orthogonal indexer (pyfive/zarr semantics), attribute and filter
mapping (active.py:126-159, hdf2numcodec.py:4-89)."""
import numpy as np
import pytest

from pyactivestorage_amd.indexing import OrthogonalIndexer
from pyactivestorage_amd.storage import Shuffle, Zlib
from pyactivestorage_amd.variable import decode_filters, get_missing_attributes

INDEXES = [
    Ellipsis, (slice(6, 7), slice(None), slice(None)), (slice(None), slice(0, 64, 3), slice(None)),
    (slice(None), slice(None), slice(0, 128, 4)), (slice(6, 7), slice(0, 64, 3), slice(0, 128, 4)),
    (slice(1, 11, 2), slice(0, 64, 3), slice(0, 128, 4)), (slice(None), [0, 1, 5, 7, 30, 31], slice(None)),
    (slice(None), [0, 1, 5, 7, 30, 31, 50, 51, 53], slice(None)),   # test_active_axis.py:28-38
    (3, slice(2, 50), 7), (slice(None), [40, 3, 3, 17], 5), (slice(0, 12), np.arange(64) % 3 == 0, slice(None)),
]


def _assemble(arr, index, chunks):
    """Rebuild arr[index] from the indexer's per-chunk projections."""
    ix = OrthogonalIndexer(index, arr.shape, chunks)
    out = np.full(ix.shape, -1, dtype=arr.dtype)
    for coords, projs in ix:
        chunk = arr[tuple(slice(c * n, (c + 1) * n) for c, n in zip(coords, chunks))]
        sel = tuple(p.chunk_sel for p in projs)
        idx = []
        for p in projs:
            s = p.chunk_sel
            if isinstance(s, slice):
                idx.append(np.arange(s.start, s.stop, s.step))
            elif isinstance(s, np.ndarray):
                idx.append(s)
            else:
                idx.append(np.array([s]))
        block = chunk[np.ix_(*idx)]
        block = block.reshape([len(i) for i, p in zip(idx, projs) if not isinstance(p.chunk_sel, (int, np.integer))])
        where = np.ix_(*[p.out_pos for p in projs if not isinstance(p.chunk_sel, (int, np.integer))])
        out[where] = block
        del sel
    return ix, out


@pytest.mark.parametrize("k", range(len(INDEXES)))
def test_indexer_reassembles_numpy_orthogonal_selection(k):
    arr = np.arange(12 * 64 * 128).reshape(12, 64, 128)
    index = INDEXES[k]
    ix, got = _assemble(arr, index, (6, 32, 32))
    # numpy orthogonal (outer) indexing of the same selection
    norm = index if isinstance(index, tuple) else (index,)
    if norm == (Ellipsis,):
        norm = (slice(None),) * 3
    want = arr
    for d in reversed(range(3)):
        s = norm[d]
        want = np.take(want, np.arange(arr.shape[d])[s], axis=d)
    assert got.shape == want.shape == ix.shape
    assert np.array_equal(got, want)


def test_indexer_nchunks_and_drop_axes():
    ix = OrthogonalIndexer((slice(0, 5), 3, [1, 40]), (12, 64, 128), (6, 32, 32))
    assert ix.dim_indexers[0].nchunks == 2 and ix.dim_indexers[2].nchunks == 4
    assert not hasattr(ix.dim_indexers[1], "nchunks")
    assert ix.drop_axes == (1,) and ix.shape == (5, 2)
    with pytest.raises(IndexError):
        OrthogonalIndexer((slice(None, None, -1),), (12,), (6,))
    with pytest.raises(IndexError):
        OrthogonalIndexer((12,), (12,), (6,))


def test_get_missing_attributes_semantics():
    """active.py:126-159 including hfix and valid_range splitting."""
    a = {"_FillValue": np.array([-900.], dtype=np.float32), "missing_value": np.array([7.0])}
    f, m, lo, hi = get_missing_attributes(a)
    assert f == np.float32(-900.) and m == 7.0 and lo is None and hi is None
    assert not isinstance(m, np.ndarray)
    f, m, lo, hi = get_missing_attributes({"valid_range": np.array([1.0, 9.0])})
    assert (lo, hi) == (1.0, 9.0)
    with pytest.raises(ValueError, match="Invalid combination"):
        get_missing_attributes({"valid_min": 1.0, "valid_range": [1.0, 2.0]})
    m = get_missing_attributes({"missing_value": np.array([1.0, 2.0])})[1]
    assert isinstance(m, np.ndarray) and m.size == 2


def test_decode_filters_mapping():
    comp, filt = decode_filters([{"filter_id": 2, "client_data": [8]}, {"filter_id": 1, "client_data": [4]}],
                                8, "tas")
    assert isinstance(comp, Zlib) and comp.level == 4
    assert len(filt) == 1 and isinstance(filt[0], Shuffle) and filt[0].elementsize == 8
    comp, filt = decode_filters([{"filter_id": 2, "client_data": [4]}], 4, "x")  # no IndexError here
    assert comp is None and filt[0].elementsize == 4
    with pytest.raises(NotImplementedError):
        decode_filters([{"filter_id": 32001, "client_data": []}], 4, "x")
    with pytest.raises(ValueError):
        decode_filters([{"filter_id": 1, "client_data": [1]}, {"filter_id": 1, "client_data": [1]}], 4, "x")


# ---------------------------------------------------------------------------
# pyas_combine_grid tables (Active._grid_tables) vs the general segment plan
# ---------------------------------------------------------------------------
def _segments_argsort(chunk_list, axes, final_shape):
    """The general path of Active._reduce: per output, the partial indices in
    chunk order (what pyas_combine_segments folds)."""
    sizes, fidx = [], []
    for _, projs in chunk_list:
        pos = [p.out_pos if i not in axes else np.zeros(1, dtype=np.int64) for i, p in enumerate(projs)]
        grids = np.meshgrid(*pos, indexing="ij")
        fidx.append(np.ravel_multi_index([g.reshape(-1) for g in grids], final_shape))
        sizes.append(grids[0].size)
    out_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    f_all = np.concatenate(fidx)
    order = np.argsort(f_all, kind="stable")
    seg = np.searchsorted(f_all[order], np.arange(int(np.prod(final_shape)) + 1))
    return [list(order[seg[f]:seg[f + 1]]) for f in range(len(seg) - 1)]


def _segments_grid(out_off, t, axes, final_shape, nd):
    """k_combine_grid's index arithmetic restated on the host."""
    blob = t["blob"]
    n_coords = t["n_coords"]
    gstride = [int(np.prod(n_coords[d + 1:])) for d in range(nd)]
    red = [d for d in range(nd) if d in axes]
    out = []
    for f in range(int(np.prod(final_shape))):
        p = np.unravel_index(f, final_shape)
        a = [0] * nd
        j, jstride = 0, 1
        for d in reversed(range(nd)):
            if d in axes:
                continue
            a[d] = int(blob[t["pos_coord"][d] + p[d]])
            j += int(blob[t["pos_local"][d] + p[d]]) * jstride
            jstride *= int(blob[t["coord_count"][d] + a[d]])
        nk = sum(a[d] * gstride[d] for d in range(nd) if d not in axes)
        seg = []
        for layer in np.ndindex(*[n_coords[d] for d in red]):
            n = nk + sum(c * gstride[d] for c, d in zip(layer, red))
            seg.append(int(out_off[n]) + j)
        out.append(seg)
    return out


@pytest.mark.parametrize("index", [
    (slice(None), slice(None), slice(None)),
    (slice(1, 9), slice(2, 11, 2), slice(None)),
    (slice(1, 10, 3), slice(None), slice(3, 7)),
    (slice(None), [0, 5, 6, 11], slice(1, 8)),
    ([7, 1, 3], slice(None), slice(None, None, 3)),
])
@pytest.mark.parametrize("axes", [(0,), (1,), (2,), (0, 1), (0, 2), (1, 2)])
def test_grid_tables_match_segments(index, axes):
    from pyactivestorage_amd.active import Active
    from pyactivestorage_amd.indexing import OrthogonalIndexer
    shape, chunks = (10, 12, 9), (4, 5, 3)
    ix = OrthogonalIndexer(index, shape, chunks)
    chunk_list = list(ix)
    final_shape = tuple(1 if i in axes else n for i, n in enumerate(ix.shape))

    class _DS:
        ndim = 3
    act = Active.__new__(Active)
    act.ds = _DS()
    res = Active._grid_tables(act, chunk_list, axes, final_shape)
    assert res is not None
    out_off, t = res
    want = _segments_argsort(chunk_list, axes, final_shape)
    got = _segments_grid(out_off, t, axes, final_shape, 3)
    assert got == want
