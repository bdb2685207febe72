"""Batch engine: drives the HIP kernels over chunks already in device memory.

This is the MI355X replacement for the reference's per-chunk loop
(``activestorage/active.py:557-598``): instead of one ``reduce_chunk`` call
per chunk on a 30-thread pool, one launch covers every chunk of a query.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .device import Context, DeviceBuffer
from .dtypes import dtype_code, native, needs_byteswap, sum_dtype, value_class
from .masking import CompiledMask, table_layout

_CLASS_DT = {"f": "<f8", "i": "<i8", "u": "<u8"}


def partial_dtype(dt) -> np.dtype:
    """Host view of ``pyas_partial`` for storage dtype dt."""
    c = _CLASS_DT[value_class(dt)]
    return np.dtype([("sum", c), ("count", "<i8"), ("min", c), ("max", c)])


@dataclass
class Layout:
    """What every chunk of one variable shares."""
    dtype: np.dtype
    chunk_shape: tuple
    shuffle: int = 0          # fused HDF5 shuffle element size (0 = none)

    def batch_struct(self, n_chunks, data_ptr, offsets_ptr, sel_ptr=None, pool_ptr=None):
        b = _lib.Batch()
        b.dtype = dtype_code(self.dtype)
        b.byteswap = 1 if needs_byteswap(self.dtype) else 0
        b.shuffle = int(self.shuffle)
        b.ndim = len(self.chunk_shape)
        if not 1 <= b.ndim <= _lib.MAX_DIMS:
            raise NotImplementedError(f"chunk rank {b.ndim} outside 1..{_lib.MAX_DIMS}")
        for d, n in enumerate(self.chunk_shape):
            b.chunk_shape[d] = int(n)
        b.n_chunks = int(n_chunks)
        b.data = data_ptr
        b.offsets = offsets_ptr
        b.sel = sel_ptr
        b.index_pool = pool_ptr
        return b


class MaskUpload:
    """Device copy of a CompiledMask's vector tables for one selected shape."""

    def __init__(self, ctx: Context, cm: CompiledMask, sel_shape, kept, stream):
        self.struct = cm.to_struct()
        self._bufs = []
        for k, which in ((0, "_FillValue"), (1, "missing_value")):
            if cm.tables[k] is None:
                continue
            strides = table_layout(cm, k, sel_shape, "missing_value" if k == 1 else "fill")
            lo, hi, _ = cm.tables[k]
            nd = native(cm.dt)
            host = np.zeros((2, lo.size), dtype=_CLASS_DT[value_class(nd)])
            host[0] = lo
            host[1] = hi
            buf = DeviceBuffer(ctx, host.nbytes)
            ctx.h2d(buf.ptr, host, stream)
            self._bufs.append(buf)
            self.struct.tab_len[k] = lo.size
            self.struct.tab_lo[k] = buf.ptr
            self.struct.tab_hi[k] = buf.ptr + lo.size * 8
            for j, d in enumerate(kept):
                self.struct.tab_stride[k][d] = int(strides[j])

    def keepalive(self):
        return self._bufs


def reduce_chunks(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, chunk_out_ptr, total_ptr,
                  round_to_var: bool, stream) -> None:
    flags = _lib.COMBINE_ROUND_TO_VAR if round_to_var else 0
    _lib.check(ctx.lib.pyas_reduce_chunks(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                          chunk_out_ptr, total_ptr, flags, stream),
               "pyas_reduce_chunks")


def tie_chunks(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, geom: _lib.TieGeom, axes_mask: int,
               which: int, out_offsets_ptr, partials_ptr, stream) -> None:
    """NumPy's sign of every zero min (which 1) / max (which 2) among the
    chunks' partials (pyas_tie_chunks, storage.py:99-100)."""
    _lib.check(ctx.lib.pyas_tie_chunks(ctx.handle, ctypes.byref(batch), ctypes.byref(mask), ctypes.byref(geom),
                                       int(axes_mask), int(which), out_offsets_ptr, partials_ptr, stream),
               "pyas_tie_chunks")


def tie_chunks_total(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, geom: _lib.TieGeom, which: int,
                     partials_ptr, layer_base: int, lr: int, stream) -> None:
    """Level 1 of a full reduction where it can matter (pyas_tie_chunks_total):
    only the two chunks the level-2 keys can pick are scanned, so
    tie_segments afterwards gives what tie_chunks over every chunk would."""
    _lib.check(ctx.lib.pyas_tie_chunks_total(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                             ctypes.byref(geom), int(which), partials_ptr, int(layer_base),
                                             int(lr), stream),
               "pyas_tie_chunks_total")


def tie_chunk_flags(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, geom: _lib.TieGeom, axes_mask: int,
                    which: int, out_offsets_ptr, final_ptr, n_final: int, flags_ptr, stream) -> None:
    """Per chunk output: zero held / NumPy's sign, when a final min/max is a
    zero (pyas_tie_chunk_flags; for results folded in the reduce kernel)."""
    _lib.check(ctx.lib.pyas_tie_chunk_flags(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                            ctypes.byref(geom), int(axes_mask), int(which), out_offsets_ptr,
                                            final_ptr, int(n_final), flags_ptr, stream),
               "pyas_tie_chunk_flags")


def tie_grid(ctx: Context, dt, grid: _lib.Grid, parts_ptr, flags_ptr, lr: int, which: int, final_ptr,
             keys_ptr, stream) -> None:
    """NumPy's sign of the zero min/max of the `out` reduction over chunk
    layers (pyas_tie_grid, active.py:594)."""
    _lib.check(ctx.lib.pyas_tie_grid(ctx.handle, dtype_code(dt), ctypes.byref(grid), parts_ptr, flags_ptr,
                                     int(lr), int(which), final_ptr, keys_ptr, stream), "pyas_tie_grid")


def tie_segments(ctx: Context, dt, parts_ptr, index_ptr, seg_ptr, n_seg: int, n_layers: int, layer_base: int,
                 lr: int, which: int, final_ptr, keys_ptr, stream) -> None:
    """pyas_tie_segments: the level-2 sign over segment lists (or one
    output over parts[0, n_layers) when index/seg are None)."""
    _lib.check(ctx.lib.pyas_tie_segments(ctx.handle, dtype_code(dt), parts_ptr, index_ptr, seg_ptr, int(n_seg),
                                         int(n_layers), int(layer_base), int(lr), int(which), final_ptr,
                                         keys_ptr, stream), "pyas_tie_segments")


def tie_keys_reset(ctx: Context, keys_ptr, n_out: int, stream) -> None:
    _lib.check(ctx.lib.pyas_tie_keys_reset(ctx.handle, keys_ptr, int(n_out), stream), "pyas_tie_keys_reset")


def tie_finalize(ctx: Context, dt, keys_ptr, n_out: int, n_sets: int, lr: int, which: int, final_ptr,
                 stream) -> None:
    """Combine gathered keys (ranks) and write the signs (pyas_tie_finalize)."""
    _lib.check(ctx.lib.pyas_tie_finalize(ctx.handle, dtype_code(dt), keys_ptr, int(n_out), int(n_sets), int(lr),
                                         int(which), final_ptr, stream), "pyas_tie_finalize")


def reduce_axes(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, axes_mask: int, out_offsets_ptr,
                out_ptr, stream, rec: int = 0) -> None:
    """pyas_reduce_axes, or with ``rec`` (PYAS_REC_SUM/MIN/MAX) the compact
    per-output records of pyas_reduce_axes_ex."""
    _lib.check(ctx.lib.pyas_reduce_axes_ex(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                           int(axes_mask), int(rec), out_offsets_ptr, out_ptr, stream),
               "pyas_reduce_axes_ex")


def method_rec(method) -> int:
    """The record form a partial-axis query of ``method`` needs per chunk
    output (storage.py:98-100): the rounded sum for sum/mean, else the min
    or the max."""
    return {"min": _lib.REC_MIN, "max": _lib.REC_MAX}.get(method, _lib.REC_SUM)


def reduce_axes_grid(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, grid: _lib.Grid, out_ptr,
                     round_to_var: bool, stream, zero_sign: int = 0) -> None:
    """pyas_reduce_axes + pyas_combine_grid in one launch (whole chunks);
    NotImplementedError when the geometry does not admit it.  ``zero_sign``
    (1 min, 2 max): NumPy's sign of a zero result fused into the fold
    (PYAS_FOLD_ZERO_SIGN_*; the caller checks both reductions are
    elementwise)."""
    flags = (_lib.COMBINE_ROUND_TO_VAR if round_to_var else 0) | (int(zero_sign) << 8)
    _lib.check(ctx.lib.pyas_reduce_axes_grid(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                             ctypes.byref(grid), flags, out_ptr, stream),
               "pyas_reduce_axes_grid")


def select_chunks(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, out_offsets_ptr, values_ptr,
                  mask_out_ptr, stream) -> None:
    _lib.check(ctx.lib.pyas_select_chunks(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                          out_offsets_ptr, values_ptr, mask_out_ptr, stream),
               "pyas_select_chunks")


def select_scatter(ctx: Context, batch: _lib.Batch, mask: _lib.Mask, scatter: _lib.Scatter,
                   values_ptr, mask_ptr, stream) -> None:
    _lib.check(ctx.lib.pyas_select_scatter(ctx.handle, ctypes.byref(batch), ctypes.byref(mask),
                                           ctypes.byref(scatter), values_ptr, mask_ptr, stream),
               "pyas_select_scatter")


def combine_partials(ctx: Context, dt, in_ptr, n, out_ptr, round_to_var: bool, stream) -> None:
    flags = _lib.COMBINE_ROUND_TO_VAR if round_to_var else 0
    _lib.check(ctx.lib.pyas_combine_partials(ctx.handle, dtype_code(dt), in_ptr, int(n), flags,
                                             out_ptr, stream), "pyas_combine_partials")


def combine_segments(ctx: Context, dt, in_ptr, index_ptr, seg_ptr, n_seg, out_ptr, round_to_var: bool,
                     stream, rec: int = 0) -> None:
    flags = (_lib.COMBINE_ROUND_TO_VAR if round_to_var else 0) | _lib.combine_rec(rec)
    _lib.check(ctx.lib.pyas_combine_segments(ctx.handle, dtype_code(dt), in_ptr, index_ptr, seg_ptr,
                                             int(n_seg), flags, out_ptr, stream),
               "pyas_combine_segments")


def combine_grid(ctx: Context, dt, in_ptr, grid: _lib.Grid, out_ptr, round_to_var: bool, stream,
                 rec: int = 0, zero_sign: int = 0) -> None:
    """pyas_combine_grid.  ``zero_sign`` (1 min, 2 max): the records carry
    level 1's NumPy sign (PYAS_REC_ZERO_SIGN) and the combine keys level 2
    (PYAS_FOLD_ZERO_SIGN_*) over the `out` array's calls."""
    flags = (_lib.COMBINE_ROUND_TO_VAR if round_to_var else 0) | _lib.combine_rec(rec) | (int(zero_sign) << 8)
    _lib.check(ctx.lib.pyas_combine_grid(ctx.handle, dtype_code(dt), in_ptr, ctypes.byref(grid), flags,
                                         out_ptr, stream), "pyas_combine_grid")


_FORMAT = {"sum": _lib.FORMAT_SUM, "min": _lib.FORMAT_MIN, "max": _lib.FORMAT_MAX,
           "mean": _lib.FORMAT_MEAN}


def format_dtype(dt, method: str) -> np.dtype:
    """Element type pyas_format_partials writes for ``method``."""
    if method == "mean":
        return np.dtype(np.float64)
    if method == "sum":
        return native(dt) if np.dtype(dt).kind == "f" else sum_dtype(dt)
    return native(dt)


def format_partials(ctx: Context, dt, in_ptr, n, method: str, values_ptr, mask_ptr, counts_ptr,
                    stream) -> None:
    """Device form of ``Active._format`` (active.py:591-630) over n partials."""
    _lib.check(ctx.lib.pyas_format_partials(ctx.handle, dtype_code(dt), in_ptr, int(n), _FORMAT[method],
                                            values_ptr, mask_ptr, counts_ptr, stream),
               "pyas_format_partials")


def unshuffle(ctx: Context, src_ptr, dst_ptr, nbytes, elementsize, stream) -> None:
    _lib.check(ctx.lib.pyas_unshuffle(ctx.handle, src_ptr, dst_ptr, int(nbytes), int(elementsize),
                                      stream), "pyas_unshuffle")


def unshuffle_chunks(ctx: Context, src_ptr, src_offsets_ptr, dst_ptr, dst_offsets_ptr, n_chunks,
                     chunk_bytes, elementsize, stream) -> None:
    """Batched device un-shuffle of whole chunks (offset arrays on the device)."""
    _lib.check(ctx.lib.pyas_unshuffle_chunks(ctx.handle, src_ptr, src_offsets_ptr, dst_ptr, dst_offsets_ptr,
                                             int(n_chunks), int(chunk_bytes), int(elementsize), stream),
               "pyas_unshuffle_chunks")
