"""Normalise a NumPy ``chunk_selection`` into per-dimension device descriptors.

Reference: ``activestorage/storage.py:95`` (``chunk[chunk_selection]``); the
selections come from pyfive's orthogonal indexer (``active.py:465,561``):
tuples of slices, integers (dropping the axis) and 1-D integer arrays (list
indices, ``tests/unit/test_active_axis.py:37-38``), or ``np.ix_``-style
arrays for orthogonal multi-list selection.

Each chunk dimension becomes ``(start, step, count)`` with step != 0 for a
slice (any sign) or step == 0 plus ``count`` indices in an index pool.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass
class DimSel:
    start: int          # first index (slice) or pool offset (list, filled later)
    step: int           # 0 => listed indices
    count: int
    dropped: bool       # integer index: the axis disappears from the result
    indices: np.ndarray | None = None   # listed indices (step == 0)


@dataclass
class ChunkSel:
    dims: list
    shape: tuple        # shape of chunk[chunk_selection]
    kept: tuple         # chunk dims present in the result, in order

    @property
    def n_selected(self) -> int:
        n = 1
        for d in self.dims:
            n *= d.count
        return n

    def is_full(self, chunk_shape) -> bool:
        return all(d.step == 1 and d.start == 0 and d.count == n and not d.dropped
                   for d, n in zip(self.dims, chunk_shape))


def _int_index(i, n, axis):
    i = int(i)
    if i < -n or i >= n:
        raise IndexError(f"index {i} is out of bounds for axis {axis} with size {n}")
    return i + n if i < 0 else i


def _as_index_array(x, n, axis):
    a = np.asarray(x)
    if a.dtype == bool:
        if a.shape != (n,):
            raise IndexError(f"boolean index did not match indexed array along axis {axis}; "
                             f"size of axis is {n} but size of corresponding boolean axis is {a.size}")
        return np.nonzero(a)[0].astype(np.int64)
    if a.dtype.kind not in "iu":
        raise IndexError("arrays used as indices must be of integer (or boolean) type")
    a = a.astype(np.int64).reshape(-1)
    bad = (a < -n) | (a >= n)
    if bad.any():
        raise IndexError(f"index {int(a[bad][0])} is out of bounds for axis {axis} with size {n}")
    return np.where(a < 0, a + n, a)


def normalize(chunk_selection, shape) -> ChunkSel:
    shape = tuple(int(s) for s in shape)
    ndim = len(shape)
    sel = chunk_selection if isinstance(chunk_selection, tuple) else (chunk_selection,)
    # expand Ellipsis
    n_ell = sum(1 for s in sel if s is Ellipsis)
    if n_ell > 1:
        raise IndexError("an index can only have a single ellipsis ('...')")
    if any(s is None for s in sel):
        raise NotImplementedError("np.newaxis in a chunk selection is not supported")
    n_real = len(sel) - n_ell
    if n_real > ndim:
        raise IndexError(f"too many indices for array: array is {ndim}-dimensional, "
                         f"but {n_real} were indexed")
    if n_ell:
        k = [i for i, x in enumerate(sel) if x is Ellipsis][0]
        sel = sel[:k] + (slice(None),) * (ndim - n_real) + sel[k + 1:]
    else:
        sel = sel + (slice(None),) * (ndim - n_real)

    adv = [d for d, s in enumerate(sel)
           if isinstance(s, list) or (isinstance(s, np.ndarray) and s.ndim > 0)]
    if len(adv) > 1:
        # only np.ix_-style (orthogonal) multi-array selections are supported
        ok = True
        for j, d in enumerate(adv):
            a = np.asarray(sel[d])
            if a.ndim != len(adv) or sum(1 for x in a.shape if x != 1) > 1 or \
                    (a.size > 1 and a.shape[j] != a.size):
                ok = False
        if not ok or adv != list(range(adv[0], adv[0] + len(adv))):
            raise NotImplementedError("vectorised (non-orthogonal) fancy indexing of a chunk "
                                      "is not supported")

    if len(adv) == 1 and np.asarray(sel[adv[0]]).ndim > 1:
        raise NotImplementedError("multi-dimensional index arrays in a chunk selection "
                                  "are not supported")

    dims, out_shape, kept = [], [], []
    for d, (s, n) in enumerate(zip(sel, shape)):
        if isinstance(s, np.ndarray) and s.ndim == 0 and s.dtype.kind in "iu":
            s = int(s)
        if isinstance(s, slice):
            start, stop, step = s.indices(n)
            cnt = len(range(start, stop, step))
            dims.append(DimSel(start if cnt else 0, step, cnt, False))
            out_shape.append(cnt)
            kept.append(d)
        elif isinstance(s, (list, np.ndarray)):
            idx = _as_index_array(s, n, d)
            if idx.size == 0:
                dims.append(DimSel(0, 1, 0, False))
            else:
                dims.append(DimSel(0, 0, int(idx.size), False, idx))
            out_shape.append(int(idx.size))
            kept.append(d)
        elif isinstance(s, (int, np.integer)):
            dims.append(DimSel(_int_index(s, n, d), 1, 1, True))
        else:
            raise IndexError("only integers, slices (`:`), ellipsis (`...`), numpy.newaxis "
                             "(`None`) and integer or boolean arrays are valid indices")
    return ChunkSel(dims, tuple(out_shape), tuple(kept))


def pack(selections, ndim):
    """Pack per-chunk ChunkSel objects into the ABI's int32 (n, MAX_DIMS, 3)
    table plus the int32 index pool."""
    n = len(selections)
    table = np.zeros((n, _lib.MAX_DIMS, 3), dtype=np.int32)
    table[:, :, 1] = 1
    table[:, :, 2] = 1
    pool_parts, pos = [], 0
    for c, cs in enumerate(selections):
        for d, ds in enumerate(cs.dims):
            if ds.step == 0:
                table[c, d] = (pos, 0, ds.count)
                pool_parts.append(ds.indices.astype(np.int32))
                pos += ds.count
            else:
                table[c, d] = (ds.start, ds.step, ds.count)
    pool = np.concatenate(pool_parts) if pool_parts else np.zeros(1, dtype=np.int32)
    return table, pool
