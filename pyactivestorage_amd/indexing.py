"""Orthogonal chunk indexer (host planning for ``Active.__getitem__``).

The reference builds ``pyfive.indexing.OrthogonalIndexer(index, ZarrArrayStub(shape,
chunks))`` (``activestorage/active.py:451,465``) and iterates it for
``(chunk_coords, chunk_selection, out_selection)`` (``active.py:561``).  pyfive
1.1.2 is absent from the image; this restates the published (zarr v2 derived)
algorithm per dimension:

* integer  -> one chunk, in-chunk integer, the axis is dropped (no ``nchunks``:
  ``Active`` refuses reductions, ``active.py:491-500``);
* slice (step >= 1) -> every chunk the range touches, in-chunk slice starting at
  the first selected element, contiguous output range;
* integer array / list / bool mask -> grouped by chunk, in-chunk index arrays,
  output positions (any order, duplicates allowed);
* ``nchunks`` of a dimension is ceil(dim_len / chunk_len), the total number
  of chunks along it (used to size ``out`` along reduced axes, active.py:502-507).

Unlike zarr, selections are returned as explicit per-dimension objects
(:class:`DimProjection`) rather than ``np.ix_`` tuples, so the planner never
depends on NumPy's mixed advanced-indexing rules.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass

import numpy as np


def _ceildiv(a, b):
    return -(-a // b)


@dataclass
class DimProjection:
    chunk_ix: int
    chunk_sel: object        # int, slice, or int64 ndarray of in-chunk indices
    out_pos: np.ndarray      # output positions along this dim (empty for dropped)


class _IntDim:
    kind = "int"

    def __init__(self, sel, dim_len, chunk_len):
        sel = int(sel)
        if sel < 0:
            sel += dim_len
        if not 0 <= sel < dim_len:
            raise IndexError(f"index out of bounds for dimension with length {dim_len}")
        self.sel, self.dim_len, self.chunk_len = sel, dim_len, chunk_len
        self.nitems = 1

    def __iter__(self):
        ix = self.sel // self.chunk_len
        yield DimProjection(ix, self.sel - ix * self.chunk_len, np.zeros(0, dtype=np.int64))


class _SliceDim:
    kind = "slice"

    def __init__(self, sel, dim_len, chunk_len):
        self.start, self.stop, self.step = sel.indices(dim_len)
        if self.step < 1:
            raise IndexError("only slices with step >= 1 are supported")
        self.dim_len, self.chunk_len = dim_len, chunk_len
        self.nitems = max(0, _ceildiv(self.stop - self.start, self.step))
        self.nchunks = _ceildiv(dim_len, chunk_len)

    def __iter__(self):
        if self.nitems == 0:
            return
        for ix in range(self.start // self.chunk_len, _ceildiv(self.stop, self.chunk_len)):
            off = ix * self.chunk_len
            lim = min(self.dim_len, off + self.chunk_len)
            if self.start < off:
                rem = (off - self.start) % self.step
                first = (self.step - rem) if rem else 0
                out0 = _ceildiv(off - self.start, self.step)
            else:
                first = self.start - off
                out0 = 0
            last = (lim - off) if self.stop > lim else (self.stop - off)
            n = max(0, _ceildiv(last - first, self.step))
            if n == 0:
                continue
            yield DimProjection(ix, slice(first, last, self.step),
                                np.arange(out0, out0 + n, dtype=np.int64))


class _ArrayDim:
    kind = "array"

    def __init__(self, sel, dim_len, chunk_len):
        a = np.asarray(sel)
        if a.dtype == bool:
            if a.shape != (dim_len,):
                raise IndexError("boolean index length does not match the dimension")
            a = np.nonzero(a)[0]
        if a.ndim != 1 or a.dtype.kind not in "iu":
            raise IndexError("integer arrays used as indices must be 1-D")
        a = a.astype(np.int64)
        a = np.where(a < 0, a + dim_len, a)
        if ((a < 0) | (a >= dim_len)).any():
            raise IndexError(f"index out of bounds for dimension with length {dim_len}")
        self.sel, self.dim_len, self.chunk_len = a, dim_len, chunk_len
        self.nitems = a.size
        self.nchunks = _ceildiv(dim_len, chunk_len)

    def __iter__(self):
        ch = self.sel // self.chunk_len
        order = np.argsort(ch, kind="stable")
        for ix in np.unique(ch):
            pos = order[ch[order] == ix]
            yield DimProjection(int(ix), self.sel[pos] - ix * self.chunk_len, pos.astype(np.int64))


def _normalize(index, ndim):
    sel = index if isinstance(index, tuple) else (index,)
    if sum(1 for s in sel if s is Ellipsis) > 1:
        raise IndexError("an index can only have a single ellipsis ('...')")
    n_real = sum(1 for s in sel if s is not Ellipsis)
    if n_real > ndim:
        raise IndexError(f"too many indices for array with {ndim} dimensions")
    ell = [i for i, s in enumerate(sel) if s is Ellipsis]
    if ell:
        k = ell[0]
        sel = sel[:k] + (slice(None),) * (ndim - n_real) + sel[k + 1:]
    return sel + (slice(None),) * (ndim - len(sel))


class OrthogonalIndexer:
    """Iterates ``(chunk_coords, [DimProjection per dim])`` over every chunk the
    orthogonal selection touches (C order of chunk coordinates)."""

    def __init__(self, index, shape, chunks):
        self.array_shape = tuple(int(s) for s in shape)
        self.chunks = tuple(int(c) for c in chunks)
        sel = _normalize(index, len(self.array_shape))
        dims = []
        for s, n, c in zip(sel, self.array_shape, self.chunks):
            if isinstance(s, slice):
                dims.append(_SliceDim(s, n, c))
            elif isinstance(s, (list, np.ndarray)) and np.ndim(s) > 0:
                dims.append(_ArrayDim(s, n, c))
            elif isinstance(s, (int, np.integer)) or (isinstance(s, np.ndarray) and s.ndim == 0):
                dims.append(_IntDim(s, n, c))
            else:
                raise IndexError(f"unsupported selection {s!r}")
        self.dim_indexers = dims
        self.shape = tuple(d.nitems for d in dims if d.kind != "int")
        self.drop_axes = tuple(i for i, d in enumerate(dims) if d.kind == "int")

    def __iter__(self):
        for projs in itertools.product(*self.dim_indexers):
            yield tuple(p.chunk_ix for p in projs), list(projs)
