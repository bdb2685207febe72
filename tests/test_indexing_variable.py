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
