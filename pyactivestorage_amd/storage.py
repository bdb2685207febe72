"""Drop-in replacement for ``activestorage/storage.py`` backed by the MI355X.

``reduce_chunk`` keeps the reference signature, argument meaning, return
types and error behaviour (``activestorage/storage.py:8-104``), so it can be
patched in exactly where the reference is called by name::

    import activestorage.active, pyactivestorage_amd.storage as gpu
    activestorage.active.reduce_chunk = gpu.reduce_chunk      # active.py:20,765

Per chunk the host reads the bytes (``read_block``, storage.py:156-162) and
undoes compression (zlib, storage.py:119-120; GPU inflate is a later row);
everything else — HDF5 byte-unshuffle, byte order, hyperslab selection,
``_FillValue``/``missing_value``/``valid_min``/``valid_max`` masking and the
sum/min/max/mean/count reduction — runs in one fused HIP kernel.  There is no
CPU fallback: without the HIP library or a GPU this raises ``RuntimeError``.

For throughput use :mod:`pyactivestorage_amd.active` / :mod:`.batch`, which
reduce every chunk of a query in one launch from device-resident memory.
"""
from __future__ import annotations

import ctypes
import os
import threading
import zlib

import numpy as np

from . import _lib, engine, results, selection, zerosign
from .device import get_context
from .dtypes import dtype_code, native, needs_byteswap, sum_dtype
from .inflate import inflate_chunk, is_zlib
from .masking import compile_missing

try:   # CPython hot path of the coalesced drop-in (built by csrc/Makefile)
    from . import _fastpath
except ImportError:   # pragma: no cover - planning stays in Python, still on the GPU
    _fastpath = None

__all__ = ["reduce_chunk", "reduce_opens3_chunk", "reduce_chunk_bytes", "filter_pipeline",
           "read_block", "Shuffle", "Zlib"]


class Zlib:
    """Minimal stand-in for ``numcodecs.Zlib`` (hdf2numcodec.py:34-35)."""

    codec_id = "zlib"

    def __init__(self, level=1):
        self.level = level

    def decode(self, buf, out=None):
        return zlib.decompress(bytes(buf))


class Shuffle:
    """Marker for ``numcodecs.Shuffle`` (hdf2numcodec.py:36-37); decoded on the GPU."""

    codec_id = "shuffle"

    def __init__(self, elementsize=4):
        self.elementsize = int(elementsize)


def read_block(open_file, offset, size):
    """``storage.py:156-162``: positioned read restoring the cursor."""
    place = open_file.tell()
    open_file.seek(offset)
    data = open_file.read(size)
    open_file.seek(place)
    return data


def _decompress(chunk, compression):
    """Host ingest: undo compression (``storage.py:119-120``)."""
    if compression is None:
        return chunk
    if getattr(compression, "codec_id", None) == "zlib":
        return zlib.decompress(bytes(chunk))
    return compression.decode(chunk)


def _shuffle_sizes(filters):
    """Element sizes of the shuffle filters, in application (reverse) order."""
    out = []
    for f in reversed(list(filters or [])):
        if getattr(f, "codec_id", None) != "shuffle":
            raise NotImplementedError(
                f"filter {f!r} is not supported by the MI355X backend (only the HDF5 "
                "shuffle filter, hdf2numcodec.py:36-37)")
        out.append(int(f.elementsize))
    return out


def filter_pipeline(chunk, compression, filters):
    """Host half of ``storage.py:107-123``: decompression only.  The shuffle
    filters are reversed on the device inside :func:`reduce_chunk_bytes`."""
    _shuffle_sizes(filters)  # validates
    return _decompress(chunk, compression)


def _normalize_axes(axis, ndim):
    if axis is None:
        return tuple(range(ndim))
    if isinstance(axis, (int, np.integer)):
        axis = (axis,)
    out = []
    for a in axis:
        a = int(a)
        if a < -ndim or a >= ndim:
            raise np.exceptions.AxisError(a, ndim)
        out.append(a % ndim)
    if len(set(out)) != len(out):
        raise ValueError("duplicate value in 'axis'")
    return tuple(out)


def reduce_chunk(rfile, offset, size, compression, filters, missing, dtype, shape, order,
                 chunk_selection, axis, method=None, option_disable_chunk_cache=False):
    """GPU ``reduce_chunk`` (``activestorage/storage.py:8-104``).

    Returns ``(tmp, N)`` exactly like the reference: ``tmp`` is
    ``method(chunk[chunk_selection] masked, axis, keepdims=True)`` and ``N``
    the count of unmasked elements, or ``(selected masked data, None)`` when
    ``method`` is None.
    """
    if COALESCE and method is not None:
        # 1. a call shape seen before: planned, run and formatted in C
        #    (pyas_fastpath.cpp -> pyas_coalesced_reduce)
        if _fastpath is not None:
            r = _fastpath.reduce(rfile, offset, size, compression, filters, missing, dtype, shape,
                                 order, chunk_selection, axis, method)
            if r is not None:
                return r
        # 2. plan it here (and register the plan with the C path)
        if rfile.__class__ is str or isinstance(rfile, (bytes, os.PathLike)):
            r = _coalesced(rfile, offset, size, compression, filters, missing, dtype, shape, order,
                           chunk_selection, axis, method)
            if r is not None:
                return r
    if hasattr(rfile, "id") and hasattr(rfile.id, "_get_raw_chunk"):
        # pyfive.high_level.Dataset branch (storage.py:88-91)
        class _StoreInfo:
            pass
        info = _StoreInfo()
        info.byte_offset, info.size = offset, size
        raw = rfile.id._get_raw_chunk(info)
    else:
        try:
            with open(rfile, "rb") as fh:
                raw = _read_pinned(fh, offset, size)
        except FileNotFoundError:
            # storage.py:63-76 falls back to an HTTP(S) read through fsspec
            import fsspec  # optional dependency of the reference
            fs = fsspec.filesystem("http")
            with fs.open(rfile, "rb") as fh:
                raw = read_block(fh, offset, size)
    return reduce_chunk_bytes(raw, compression, filters, missing, dtype, shape, order,
                              chunk_selection, axis, method)


# ---------------------------------------------------------------------------
# coalesced per-chunk path (pyas_coalesced_reduce)
# ---------------------------------------------------------------------------
# The reference's pool calls reduce_chunk with the same dtype / shape /
# filters / missing objects for every chunk of a query (active.py:556-589),
# so everything but the byte range is planned once and looked up by the
# identity of those objects (the entry keeps them alive and re-checks `is`).
COALESCE = os.environ.get("PYAS_COALESCE", "1") != "0"
# PYAS_PERCALL_INFLATE=device: the per-call path inflates zlib chunks with
# pyas_inflate instead of zlib on the calling thread
PERCALL_DEVICE_INFLATE = os.environ.get("PYAS_PERCALL_INFLATE", "host") == "device"
_PLAN_CAP = 256
_plans: dict = {}
_plan_lock = threading.Lock()


class _Layout:
    """Per (dtype, shape, order, filters, compression, missing): the
    pyas_chunk_desc / pyas_mask pair and the per-(selection, axis) plans."""

    __slots__ = ("refs", "ok", "dt", "pdt", "cm", "mask", "mask_ref", "desc_base", "rev", "shape",
                 "zlib", "sels", "order")

    def __init__(self, refs, compression, filters, missing, dtype, shape, order):
        self.refs = refs
        self.ok = False
        self.sels = {}
        dt = self.dt = np.dtype(dtype)
        self.shape = shape
        self.order = order
        if order not in ("C", "F") or dt.kind not in "iuf":
            return
        try:
            shuffles = _shuffle_sizes(filters)
        except NotImplementedError:
            return
        fused = 0
        if shuffles:
            if len(shuffles) != 1 or shuffles[0] != dt.itemsize:
                return                          # a standalone un-shuffle pass: per-call path
            fused = dt.itemsize if dt.itemsize > 1 else 0
        self.zlib = is_zlib(compression)
        if compression is not None and not self.zlib:
            return
        try:
            cm = self.cm = compile_missing(missing, dt)
        except Exception:
            return                              # the per-call path raises it
        if cm.tables[0] is not None or cm.tables[1] is not None:
            return                              # vector mask tables: per-call path
        self.rev = order == "F" and len(shape) > 1
        dev_shape = shape[::-1] if self.rev else shape
        if not 1 <= len(shape) <= _lib.MAX_DIMS:
            return
        self.mask = cm.to_struct()
        self.mask_ref = ctypes.byref(self.mask)
        d = self.desc_base = _lib.ChunkDesc()
        d.dtype = dtype_code(dt)
        d.byteswap = 1 if needs_byteswap(dt) else 0
        d.shuffle = fused
        d.ndim = len(shape)
        for i, n in enumerate(dev_shape):
            d.chunk_shape[i] = int(n)
        d.zlib = 1 if self.zlib else 0
        self.pdt = engine.partial_dtype(dt)
        self.ok = True

    def plan(self, chunk_selection, axis, which=0):
        """(desc, sel_ptr, pool_ptr, pool_len, n_out, keep_shape, n_red, n_sel,
        keepalive) for one selection + axis (+ the min (1) / max (2) whose
        zero sign the batch fixes, pyas_tie_chunks), cached when the
        selection is made of slices (what pyfive's indexer produces)."""
        sel = chunk_selection if chunk_selection.__class__ is tuple else (chunk_selection,)
        try:   # slices only (ints, lists and arrays have no .start): cacheable
            key = (tuple([(s.start, s.stop, s.step) for s in sel]),
                   axis if axis is None or axis.__class__ is int else tuple(axis), which)
        except (AttributeError, TypeError):
            key = None
        if key is not None:
            hit = self.sels.get(key)
            if hit is not None:
                return hit
        shape = self.shape
        cs = selection.normalize(chunk_selection, shape)
        axes = _normalize_axes(axis, len(cs.shape))
        rev = self.rev
        nd = len(shape)
        dev_of = (lambda k: nd - 1 - k) if rev else (lambda k: k)
        mask_bits = 0
        for i in axes:
            mask_bits |= 1 << dev_of(cs.kept[i])
        for k, ds in enumerate(cs.dims):   # integer-indexed dims are reduced too (extent 1)
            if ds.dropped:
                mask_bits |= 1 << dev_of(k)
        keep_shape = tuple(1 if i in axes else n for i, n in enumerate(cs.shape))
        n_out = 1
        for i, n in enumerate(cs.shape):
            if i not in axes:
                n_out *= n
        n_red = 1
        for i in axes:
            n_red *= cs.shape[i]
        desc = _lib.ChunkDesc()
        ctypes.pointer(desc)[0] = self.desc_base
        desc.axes_mask = mask_bits
        if which and self.dt.kind == "f":
            desc.tie_which = which
            desc.tie = zerosign.geometry(shape, self.order, cs, self.cm.masked, self.dt)
        dev_dims = cs.dims[::-1] if rev else cs.dims
        full = all(ds.step == 1 and ds.start == 0 and ds.count == n and not ds.dropped
                   for ds, n in zip(dev_dims, shape[::-1] if rev else shape))
        if full:
            table = pool = None
            sel_ptr = pool_ptr = None
            pool_len = 0
        else:
            table, pool = selection.pack([selection.ChunkSel(dev_dims, cs.shape, cs.kept)], nd)
            table = np.ascontiguousarray(table.reshape(-1), dtype=np.int32)
            pool = np.ascontiguousarray(pool, dtype=np.int32)
            sel_ptr, pool_ptr, pool_len = table.ctypes.data, pool.ctypes.data, int(pool.size)
        ent = (desc, ctypes.byref(desc), sel_ptr, pool_ptr, pool_len, n_out, keep_shape, n_red,
               cs.n_selected, (table, pool))
        if key is not None:
            if len(self.sels) > 4096:
                self.sels.clear()
            self.sels[key] = ent
        return ent


def _layout(compression, filters, missing, dtype, shape, order):
    if shape.__class__ is not tuple:
        shape = tuple(shape) if isinstance(shape, list) else (shape,)
    fkey = None if filters is None else tuple([(f.__class__, getattr(f, "elementsize", None))
                                               for f in filters])
    key = (id(missing), id(dtype), id(compression), fkey, shape, order)
    lay = _plans.get(key)
    if lay is not None and lay.refs[0] is missing and lay.refs[1] is dtype and \
            lay.refs[2] is compression:
        return lay
    shape = tuple(int(s) for s in shape)
    lay = _Layout((missing, dtype, compression), compression, filters, missing, dtype, shape, order)
    with _plan_lock:
        if len(_plans) >= _PLAN_CAP:
            _plans.clear()
        _plans[key] = lay
    return lay


def _coalesced(rfile, offset, size, compression, filters, missing, dtype, shape, order,
               chunk_selection, axis, method):
    """The per-chunk call through pyas_coalesced_reduce, or None when this
    call must take the per-call path (which then raises the reference's
    exact exception for bad input)."""
    try:
        kind, is_ma = results.METHODS.get(method) or results.method_kind(method)
        lay = _layout(compression, filters, missing, dtype, shape, order)
        if not lay.ok:
            return None
        desc, desc_ref, sel_ptr, pool_ptr, pool_len, n_out, keep_shape, n_red, n_sel, _ = \
            lay.plan(chunk_selection, axis, _TIE_WHICH.get(kind, 0))
    except Exception:
        return None
    if n_out == 0 or n_sel == 0:
        return None
    ctx = _ctx0 or _get_ctx0()
    if n_out == 1:
        # per-thread landing buffer for the one partial (+ info), reused
        tb = getattr(_tls, "one", None)
        if tb is None:
            raw = np.zeros(64, dtype=np.uint8)
            tb = _tls.one = (raw, raw.ctypes.data,
                             (ctypes.c_int64 * 3).from_address(raw.ctypes.data + 32), {})
        out_ptr, info = tb[1], tb[2]
    else:
        out = np.empty(n_out, dtype=lay.pdt)
        out_ptr = out.ctypes.data
        info = (ctypes.c_int64 * 3)()
    rc = _reduce_fn(ctx._coalescer or ctx.coalescer(),
                    rfile.encode("utf-8", "surrogateescape") if rfile.__class__ is str else os.fsencode(rfile),
                    int(offset), int(size), desc_ref, lay.mask_ref, sel_ptr, pool_ptr, pool_len, n_out,
                    out_ptr, info)
    if rc != _lib.OK:
        if rc in (_lib.EIO, _lib.ENOTSUP, _lib.EINDEX, _lib.EINVAL):
            return None
        _lib.check(rc, "pyas_coalesced_reduce")
    if n_out == 1:
        if _fastpath is not None and kind != "mean":
            _register_fast(lay, compression, filters, missing, dtype, shape, order, chunk_selection,
                           axis, method, kind, is_ma, keep_shape, n_sel)
        view = tb[3].get(lay.pdt)
        if view is None:
            view = tb[3][lay.pdt] = tb[0][:32].view(lay.pdt)
        return results.build_one(view[0], keep_shape, kind, is_ma, lay.dt, lay.cm.masked, n_red,
                                 n_sel)
    if lay.rev:
        parts = out.reshape(keep_shape[::-1]).transpose()
    else:
        parts = out.reshape(keep_shape)
    return results.build(parts, kind, is_ma, lay.dt, lay.cm.masked, n_red, n_sel)


_tls = threading.local()
_ctx0 = None
_reduce_fn = None


def _get_ctx0():
    global _ctx0, _reduce_fn
    ctx = get_context(0)
    _reduce_fn = ctx.lib.pyas_coalesced_reduce
    if _fastpath is not None:
        _fastpath.bind(ctypes.cast(_reduce_fn, ctypes.c_void_p).value, ctx.coalescer(),
                       np.ma.MaskedArray)
    _ctx0 = ctx
    return ctx


_KIND = {"sum": 0, "min": 1, "max": 2}
_TIE_WHICH = {"min": 1, "max": 2}
_VCLASS = {"f": 0, "i": 1, "u": 2}


def _register_fast(lay, compression, filters, missing, dtype, shape, order, chunk_selection, axis,
                   method, kind, is_ma, keep_shape, n_sel):
    """Hand one call shape's plan to the C hot path (pyas_fastpath.cpp)."""
    desc, _, sel_ptr, _, pool_len, _, _, _, _, (table, pool) = lay.plan(chunk_selection, axis,
                                                                        _TIE_WHICH.get(kind, 0))
    if not keep_shape:
        return
    rdt = sum_dtype(lay.dt) if kind == "sum" else native(lay.dt)
    _fastpath.register(missing, dtype, compression, filters, shape, order, chunk_selection, axis,
                       method, bytes(desc), bytes(lay.mask),
                       None if table is None else table.tobytes(),
                       b"" if pool is None or not pool_len else pool.tobytes(),
                       len(keep_shape), _KIND[kind], bool(is_ma), bool(lay.cm.masked), int(n_sel),
                       _VCLASS[lay.dt.kind], rdt.num)


def _read_pinned(fh, offset, size):
    """read_block (storage.py:156-162) into the calling thread's pinned
    staging buffer (the chunk's H2D copy is then DMA).  The view is valid
    until this thread's next call; reduce_chunk_bytes synchronizes before
    returning.  A short read (past the end of the file) returns the bytes
    that exist, as ``fh.read`` does."""
    ctx = get_context(0)
    try:   # never pin more than the file can return
        size = max(0, min(int(size), os.fstat(fh.fileno()).st_size - int(offset)))
    except (OSError, AttributeError, ValueError):
        pass
    host = ctx.thread_host_buffer(int(size))
    fh.seek(offset)
    n = fh.readinto(memoryview(host)[: int(size)])
    return memoryview(host)[: n or 0]


def reduce_opens3_chunk(fh, offset, size, compression, filters, missing, dtype, shape, order,
                        chunk_selection, axis, method=None):
    """``storage.py:165-202``: same reduction for an already-open handle."""
    fh.seek(offset)
    raw = fh.read(size)
    return reduce_chunk_bytes(raw, compression, filters, missing, dtype, shape, order,
                              chunk_selection, axis, method)


class _Sized:
    """Size stand-in for a chunk that only exists on the device."""

    def __init__(self, size):
        self.size = int(size)


def reduce_chunk_bytes(raw, compression, filters, missing, dtype, shape, order,
                       chunk_selection, axis, method=None, device=0):
    """The reduction of :func:`reduce_chunk` for chunk bytes already in memory."""
    dt = np.dtype(dtype)
    shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
    if order not in ("C", "F"):
        raise NotImplementedError(f"order={order!r}")
    shuffles = _shuffle_sizes(filters)
    ctx = get_context(device)
    st = ctx.thread_stream()
    n_expect = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    device_inflated = is_zlib(compression) and PERCALL_DEVICE_INFLATE
    if device_inflated:
        # f3: upload the deflated bytes, inflate on the device (raises like zlib)
        data = ctx.thread_buffer("data", max(n_expect, 16))
        inflate_chunk(ctx, raw, data.ptr, n_expect, st)
        buf = _Sized(n_expect)
    else:
        # one stream per call: zlib on this thread (GIL released) beats one
        # device wave per stream (~55 MB/s); the device reduces
        buf = np.frombuffer(memoryview(_decompress(raw, compression)), dtype=np.uint8)
    # .view(dtype) then .reshape(shape) errors (storage.py:59-62)
    if buf.size % dt.itemsize:
        raise ValueError("When changing to a larger dtype, its size must be a divisor of the "
                         "total size in bytes of the last axis of the array.")
    n_elem = buf.size // dt.itemsize
    if n_elem != int(np.prod(shape, dtype=np.int64)):
        raise ValueError(f"cannot reshape array of size {n_elem} into shape {shape}")

    cs = selection.normalize(chunk_selection, shape)
    rev = order == "F" and len(shape) > 1
    dev_shape = shape[::-1] if rev else shape
    dev_dims = cs.dims[::-1] if rev else cs.dims
    dev_of = (lambda d: len(shape) - 1 - d) if rev else (lambda d: d)

    if not device_inflated:
        data = ctx.thread_buffer("data", max(buf.size, 16))
        ctx.h2d(data.ptr, buf, st)
    # shuffle filters: fuse the last one when its element size is the dtype's;
    # any other shuffle pass runs as a standalone device un-shuffle first
    fused = 0
    passes = list(shuffles)
    if passes and passes[-1] == dt.itemsize:
        passes.pop()
        fused = dt.itemsize if dt.itemsize > 1 else 0
    spare = None
    for es in passes:
        if es > 1:
            if spare is None:
                spare = ctx.thread_buffer("data2", max(buf.size, 16))
            engine.unshuffle(ctx, data.ptr, spare.ptr, buf.size, es, st)
            data, spare = spare, data

    table, pool = selection.pack([selection.ChunkSel(dev_dims, cs.shape, cs.kept)], len(shape))
    # [int64 offsets[1] = {0}] [int32 sel table] [int32 index pool]
    meta = np.concatenate([np.zeros(1, dtype=np.int64).view(np.int32),
                           table.reshape(-1), pool]).astype(np.int32)
    mbuf = ctx.thread_buffer("meta", meta.nbytes)
    ctx.h2d(mbuf.ptr, meta, st)
    offsets_ptr = mbuf.ptr                    # int64 offsets[1] = {0}
    sel_ptr = mbuf.ptr + 8
    pool_ptr = sel_ptr + table.nbytes

    layout = engine.Layout(dt, dev_shape, fused)
    batch = layout.batch_struct(1, data.ptr, offsets_ptr, sel_ptr, pool_ptr)
    cm = compile_missing(missing, dt)
    mup = engine.MaskUpload(ctx, cm, cs.shape, [dev_of(d) for d in cs.kept], st)

    if not method:
        return _select(ctx, st, batch, mup, cs, dt, cm, rev), None

    kind, is_ma = results.method_kind(method)
    axes = _normalize_axes(axis, len(cs.shape))
    keep_shape = tuple(1 if i in axes else n for i, n in enumerate(cs.shape))
    n_red = 1
    for i in axes:
        n_red *= cs.shape[i]
    pdt = engine.partial_dtype(dt)
    if len(axes) == len(cs.shape):
        out = ctx.thread_buffer("out", _lib.PARTIAL_NBYTES)
        engine.reduce_chunks(ctx, batch, mup.struct, out.ptr, None, False, st)
        if kind in ("min", "max"):   # NumPy's +0.0/-0.0 when the extreme is zero
            engine.tie_chunks(ctx, batch, mup.struct, zerosign.geometry(shape, order, cs, cm.masked, dt),
                              (1 << len(shape)) - 1, 1 if kind == "min" else 2, None, out.ptr, st)
        host = np.zeros(1, dtype=pdt)
        ctx.d2h(host, out.ptr, st)
        ctx.synchronize(st)
        parts = host.reshape(keep_shape)
    else:
        chunk_axes = [dev_of(cs.kept[i]) for i in axes]
        mask_bits = 0
        for d in chunk_axes:
            mask_bits |= 1 << d
        n_out = int(np.prod(keep_shape, dtype=np.int64))
        out = ctx.thread_buffer("out", max(n_out, 1) * _lib.PARTIAL_NBYTES + 8)
        zero = np.zeros(1, dtype=np.int64)
        off_ptr = out.ptr + max(n_out, 1) * _lib.PARTIAL_NBYTES
        ctx.h2d(off_ptr, zero, st)
        if n_out:
            engine.reduce_axes(ctx, batch, mup.struct, mask_bits, off_ptr, out.ptr, st)
            if kind in ("min", "max"):
                for k, ds in enumerate(dev_dims):   # integer-indexed dims are reduced too (extent 1)
                    if ds.dropped:
                        mask_bits |= 1 << k
                engine.tie_chunks(ctx, batch, mup.struct, zerosign.geometry(shape, order, cs, cm.masked, dt),
                                  mask_bits, 1 if kind == "min" else 2, off_ptr, out.ptr, st)
        host = np.zeros(max(n_out, 1), dtype=pdt)
        ctx.d2h(host, out.ptr, st)
        ctx.synchronize(st)
        host = host[:n_out]
        if rev:
            parts = host.reshape(keep_shape[::-1]).transpose()
        else:
            parts = host.reshape(keep_shape)
    del mup
    return results.build(parts, kind, is_ma, dt, cm.masked, n_red, cs.n_selected)


def _select(ctx, st, batch, mup, cs, dt, cm, rev):
    """method=None: the masked selection itself (storage.py:95-96,102-103)."""
    n = cs.n_selected
    nd = native(dt)
    vals = np.zeros(max(n, 1), dtype=nd)
    msk = np.zeros(max(n, 1), dtype=np.uint8)
    # device layout: [int64 offsets[1]][pad to 256][values][mask bytes]
    vals_off = 256
    out = ctx.thread_buffer("out", vals_off + vals.nbytes + msk.nbytes)
    ctx.h2d(out.ptr, np.zeros(1, dtype=np.int64), st)
    if n:
        engine.select_chunks(ctx, batch, mup.struct, out.ptr, out.ptr + vals_off,
                             out.ptr + vals_off + vals.nbytes, st)
        ctx.d2h(vals, out.ptr + vals_off, st)
        ctx.d2h(msk, out.ptr + vals_off + vals.nbytes, st)
    ctx.synchronize(st)
    vals, msk = vals[:n], msk[:n].astype(bool)
    if rev:
        vals = vals.reshape(cs.shape[::-1]).transpose()
        msk = msk.reshape(cs.shape[::-1]).transpose()
    else:
        vals = vals.reshape(cs.shape)
        msk = msk.reshape(cs.shape)
    data = vals.astype(dt)  # keep the requested byte order, like chunk.view(dtype)
    if cm.masked:
        # an all-False mask is shrunk to nomask by numpy.ma.masked_where
        return np.ma.MaskedArray(data, mask=msk) if msk.any() else np.ma.MaskedArray(data)
    return data
