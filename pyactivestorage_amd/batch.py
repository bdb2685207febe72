"""Batched, device-resident chunk reduction — the throughput path.

A :class:`ReductionPlan` is everything one ``Active.__getitem__`` needs on
the device (``activestorage/active.py:476-598``): the chunk byte offsets
inside a device buffer, the per-chunk hyperslab selections, the compiled
mask, and output space for one partial per chunk plus the combined total.
Planning (host) happens once; :meth:`ReductionPlan.launch` only enqueues the
kernel chain on a stream (no host synchronisation, no allocation), so it can
be timed or captured.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib, engine, selection, zerosign
from .device import Context, DeviceBuffer
from .dtypes import native
from .masking import compile_missing


class ReductionPlan:
    """Reduce every listed chunk of one variable, fully on the device.

    Parameters
    ----------
    ctx: device context.
    dtype, chunk_shape, shuffle: the variable's storage layout.
    data_ptr: device pointer of the buffer holding the (uncompressed) chunks.
    offsets: int64 byte offsets of the chunks inside that buffer.
    selections: None (every chunk fully selected) or a list of
        :class:`selection.ChunkSel` (one per chunk, same order as offsets).
    missing: the ``(fill, missing, valid_min, valid_max)`` tuple.
    round_to_var: store per-chunk sums in the variable dtype before the
        combine, as ``Active`` does (``active.py:512,585``).
    """

    def __init__(self, ctx: Context, dtype, chunk_shape, data_ptr, offsets, *, shuffle=0,
                 selections=None, sel_table=None, index_pool=None, missing=None,
                 round_to_var=True, stream=None):
        self.ctx = ctx
        self.dtype = np.dtype(dtype)
        self.chunk_shape = tuple(int(s) for s in chunk_shape)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.n_chunks = int(offsets.size)
        es = self.dtype.itemsize
        if (offsets % es).any():
            raise ValueError("chunk offsets must be multiples of the element size")
        self.round_to_var = bool(round_to_var)
        self.cm = compile_missing(missing, self.dtype)
        self._bufs = []
        st = stream
        self.offsets_buf = self._upload(offsets, st)
        sel_ptr = pool_ptr = None
        table = None
        self.sel_table_host = None   # the uploaded selection table (host copy), None: every chunk whole
        sel_shape, kept = self.chunk_shape, tuple(range(len(self.chunk_shape)))
        self._sel0 = None        # a chunk's selection, for tie_geom
        if selections is not None:
            if len(selections) != self.n_chunks:
                raise ValueError("one selection per chunk is required")
            table, pool = selection.pack(selections, len(self.chunk_shape))
            _check_table(table, self.chunk_shape, pool)
            vector_mask = self.cm.tables[0] is not None or self.cm.tables[1] is not None
            if vector_mask or not _all_full(table, self.chunk_shape):
                # (every chunk fully selected and scalar masks: no table, the
                # kernels' lean/dense paths)
                sel_ptr = self._upload(table, st).ptr
                pool_ptr = self._upload(pool, st).ptr
                self.sel_table_host = table
            shapes = {s.shape for s in selections}
            if (self.cm.tables[0] is not None or self.cm.tables[1] is not None) and len(shapes) > 1:
                raise NotImplementedError("vector fill/missing values need equal selection shapes")
            if selections:
                sel_shape, kept = selections[0].shape, selections[0].kept
                self._sel0 = selections[0]
        elif sel_table is not None:
            # pre-packed ABI table (int32 [n, MAX_DIMS, 3]) for large planned queries
            table = np.ascontiguousarray(sel_table, dtype=np.int32)
            if table.shape != (self.n_chunks, _lib.MAX_DIMS, 3):
                raise ValueError("sel_table must have shape (n_chunks, MAX_DIMS, 3)")
            _check_table(table, self.chunk_shape, index_pool)
            if self.cm.tables[0] is not None or self.cm.tables[1] is not None:
                raise NotImplementedError("vector fill/missing values need ChunkSel selections")
            sel_ptr = self._upload(table, st).ptr
            pool_ptr = self._upload(index_pool if index_pool is not None
                                    else np.zeros(1, dtype=np.int32), st).ptr
            self.sel_table_host = table
            if self.n_chunks:
                self._sel0 = _row_sel(table[0], self.chunk_shape, index_pool)
        self.layout = engine.Layout(self.dtype, self.chunk_shape,
                                    shuffle if (shuffle and shuffle > 1 and es > 1) else 0)
        self.batch = self.layout.batch_struct(self.n_chunks, data_ptr, self.offsets_buf.ptr,
                                              sel_ptr, pool_ptr)
        self.mask_up = engine.MaskUpload(ctx, self.cm, sel_shape, kept, st)
        self.chunk_partials = DeviceBuffer(ctx, max(self.n_chunks, 1) * _lib.PARTIAL_NBYTES)
        self.total = DeviceBuffer(ctx, _lib.PARTIAL_NBYTES)

    def dense_boxes(self) -> bool:
        """Whether every chunk is whole or a unit-step box covering at least
        half of it with more than one index in its innermost dim: the chunks
        the dense per-chunk kernels walk themselves (pyas_kernels.hpp
        cut_eligible), the promise PYAS_REC_ZERO_SIGN needs."""
        r = getattr(self, "_dense_boxes", None)   # fixed per plan; replays ask every query
        if r is None:
            self._dense_class()
        return self._dense_boxes

    def no_dense_boxes(self) -> bool:
        """Whether NO chunk is whole or such a box (every chunk's selection is
        strided, listed or small): the dense launch would find nothing, so
        PYAS_REC_GENERIC_ONLY skips it."""
        if getattr(self, "_no_dense", None) is None:
            self._dense_class()
        return self._no_dense

    def _dense_class(self):
        t = self.sel_table_host
        nd = len(self.chunk_shape)
        if t is None:
            self._dense_boxes, self._no_dense = self.chunk_shape[-1] >= 2, False
            return
        step, cnt = t[:, :nd, 1], t[:, :nd, 2].astype(np.int64)
        # the kernels' cut_eligible (pyas_kernels.hpp), and chunk_is_full
        box = ((step == 1) | (cnt == 1)).all(axis=1) & (cnt >= 1).all(axis=1)
        box &= 2 * cnt.prod(axis=1) >= int(np.prod(self.chunk_shape))
        full = ((step == 1) & (cnt == np.asarray(self.chunk_shape, dtype=np.int64)[None, :])).all(axis=1)
        # DENSE_ONLY also wants more than one index in the innermost dim
        self._dense_boxes = self.chunk_shape[-1] >= 2 and bool((box & (cnt[:, nd - 1] > 1)).all())
        self._no_dense = not bool((box | full).any())

    def tie_geom(self, order="C") -> _lib.TieGeom:
        """How NumPy walks these chunks' ``chunk[sel]`` after mask_missing
        (``pyas_tie_geom``, zerosign.geometry): the zero-sign passes'
        geometry."""
        g = getattr(self, "_geom", None)
        if g is None:
            cs = self._sel0 or selection.normalize((slice(None),) * len(self.chunk_shape), self.chunk_shape)
            g = self._geom = zerosign.geometry(self.chunk_shape, order, cs, self.cm.masked, self.dtype)
        return g

    def _upload(self, arr, stream):
        arr = np.ascontiguousarray(arr)
        buf = DeviceBuffer(self.ctx, max(arr.nbytes, 16))
        self.ctx.h2d(buf.ptr, arr, stream)
        self.ctx.synchronize(stream)
        self._bufs.append(buf)
        return buf

    # ------------------------------------------------------------------
    def launch(self, stream=None, chunk_partials=True) -> None:
        """Enqueue: fused reduce of every chunk -> per-chunk partials ->
        fixed-order combine into ``self.total``."""
        out = self.chunk_partials.ptr if chunk_partials else None
        engine.reduce_chunks(self.ctx, self.batch, self.mask_up.struct, out, self.total.ptr,
                             self.round_to_var, stream)

    def total_tensor(self, torch):
        """Zero-copy torch view (32 uint8) of the device total, e.g. to hand
        it to torch.distributed (RCCL) without a copy."""
        t = getattr(self, "_total_t", None)
        if t is None:
            t = self._total_t = device_tensor(torch, self.total.ptr, _lib.PARTIAL_NBYTES,
                                              self.ctx.device)
        return t

    def read_total(self, stream=None) -> np.ndarray:
        host = np.zeros(1, dtype=engine.partial_dtype(self.dtype))
        self.ctx.d2h(host, self.total.ptr, stream)
        self.ctx.synchronize(stream)
        return host

    def read_chunk_partials(self, stream=None) -> np.ndarray:
        host = np.zeros(self.n_chunks, dtype=engine.partial_dtype(self.dtype))
        if self.n_chunks:
            self.ctx.d2h(host, self.chunk_partials.ptr, stream)
        self.ctx.synchronize(stream)
        return host


def _row_sel(row, chunk_shape, pool) -> selection.ChunkSel:
    """ChunkSel of one row of a packed selection table."""
    dims = []
    for d in range(len(chunk_shape)):
        start, step, cnt = (int(x) for x in row[d])
        if step == 0:
            dims.append(selection.DimSel(0, 0, cnt, False, np.asarray(pool[start:start + cnt], dtype=np.int64)))
        else:
            dims.append(selection.DimSel(start, step, cnt, False))
    return selection.ChunkSel(dims, tuple(d.count for d in dims), tuple(range(len(chunk_shape))))


def _all_full(table, chunk_shape) -> bool:
    """True when every chunk's selection is its whole box in C order
    (start 0, step 1, count = extent), i.e. the table can be dropped."""
    nd = len(chunk_shape)
    if table.shape[0] == 0:
        return False
    t = table[:, :nd, :]
    return bool((t[:, :, 0] == 0).all() and (t[:, :, 1] == 1).all()
                and (t[:, :, 2] == np.asarray(chunk_shape, dtype=np.int32)).all())


def _check_table(table, chunk_shape, pool):
    """Host bounds check of a packed selection table, so the device never
    reads outside a chunk (the C ABI trusts its caller)."""
    nd = len(chunk_shape)
    shape = np.array(chunk_shape + (1,) * (_lib.MAX_DIMS - nd), dtype=np.int64)
    start = table[:, :, 0].astype(np.int64)
    step = table[:, :, 1].astype(np.int64)
    cnt = table[:, :, 2].astype(np.int64)
    if (cnt < 0).any():
        raise ValueError("negative selection count")
    sl = (step != 0) & (cnt > 0)
    last = start + (cnt - 1) * step
    bad = sl & ((start < 0) | (start >= shape) | (last < 0) | (last >= shape))
    if bad.any():
        raise IndexError("selection table reaches outside the chunk")
    lst = (step == 0) & (cnt > 0)
    if lst.any():
        if pool is None:
            raise ValueError("listed selections need an index pool")
        pool = np.asarray(pool, dtype=np.int64)
        ends = start + cnt
        if (start[lst] < 0).any() or (ends[lst] > pool.size).any():
            raise IndexError("index pool reference out of range")
        dims = np.nonzero(lst)
        for c, d in zip(*dims):
            seg = pool[start[c, d]: start[c, d] + cnt[c, d]]
            if (seg < 0).any() or (seg >= shape[d]).any():
                raise IndexError("listed index outside the chunk")


def device_tensor(torch, ptr, nbytes, device):
    """Zero-copy uint8 torch tensor over a device allocation made by the C
    library (``__cuda_array_interface__``)."""
    class _Holder:
        __cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False),
                                    "version": 3, "strides": None}
    return torch.as_tensor(_Holder(), device=torch.device("cuda", device))


def finalize(total: np.ndarray, method: str, dtype, components=False, ndim=1, masked=None):
    """Host formatting of a combined partial into ``Active``'s return value
    (``active.py:591-630``): sum/min/max as the variable's reduction dtype,
    mean = sum / n (float64), or the components dict."""
    from .dtypes import sum_dtype
    dt = np.dtype(dtype)
    t = total.reshape(-1)[0]
    n = np.full((1,) * ndim, int(t["count"]), dtype=np.int64)
    shape = (1,) * ndim
    if method in ("sum", "mean"):
        # out[] holds per-chunk sums in the variable dtype, np.ma.sum(out) keeps it
        # for floats; integer out[] sums widen to int64/uint64 (active.py:594)
        rdt = native(dt) if dt.kind == "f" else sum_dtype(dt)
        val = np.full(shape, t["sum"]).astype(rdt)
    else:
        val = np.full(shape, t[method]).astype(native(dt))
    out = np.ma.MaskedArray(val, mask=np.full(shape, int(t["count"]) == 0))
    if components:
        key = "sum" if method == "mean" else method
        return {key: out, "n": n}
    if method == "mean":
        return out / n
    return out
