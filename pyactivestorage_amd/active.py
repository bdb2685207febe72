"""Batched ``Active`` front end: one device launch chain per query.

Mirrors ``activestorage/active.py``'s user API (``Active(path, ncvar)``,
``Active.method``, ``.mean()/.min()/.max(axis)``, ``.components``,
``active[index]``, ``active.py:162-427``).  The dataset is a netCDF4/HDF5
path, whose metadata and chunk index :mod:`.hdf5` reads (pyfive's part in
the reference), or a :class:`~pyactivestorage_amd.variable.ChunkedVariable`.
``__getitem__`` replaces ``_get_selection`` + ``_from_storage``
(``active.py:439-635``):

1. plan: orthogonal indexer -> per-dim projections; for box queries the
   selection table, index pool and chunk list follow by broadcasting;
2. ingest: for a file on disk, native pread threads (``max_threads``, like
   ``active.py:557``) into pinned slots copied H2D as they fill
   (``pyas_read_ranges``, row f2); zlib chunks are inflated on the device
   (``pyas_inflate``, row f3) in stream groups that overlap the reads;
   ``resident=True`` keeps decoded chunks in HBM across queries;
3. device: one fused reduce over every chunk (full-axis queries) or a
   partial-axis reduce plus the grid combine (``pyas_combine_grid``; host
   segments via ``pyas_combine_segments`` otherwise), with per-chunk sums
   rounded to the variable dtype first, like the reference's ``out`` array
   (``active.py:512,585``);
4. ``group=``: each rank of a torch.distributed group does 2-3 for its
   contiguous share of the chunks, then one all-gather and a rank-order
   device combine (row e);
5. host: format the combined partials exactly like ``active.py:591-630``.
"""
from __future__ import annotations

import concurrent.futures
import os
import threading

import warnings

import numpy as np

from . import _lib, engine, selection, zerosign
from .batch import ReductionPlan, _all_full
from .device import DeviceBuffer, get_context
from .dtypes import native, sum_dtype
from .indexing import OrthogonalIndexer
from .ingest import read_ranges, read_ranges_zlib
from .inflate import InflateBatch, is_zlib, pack_streams
from .masking import compile_missing
from .storage import _decompress, _shuffle_sizes
from .variable import ChunkedVariable, decode_filters, get_missing_attributes

_ALIGN = 256
_RESIDENT_LOCK = threading.Lock()
_RESIDENT_CV = threading.Condition(_RESIDENT_LOCK)   # slot state changes
_EMPTY, _LOADING, _LOADED = 0, 1, 2


# PYAS_AXES_FOLD=0 keeps whole-chunk box queries on the two-step path
# (pyas_reduce_axes + pyas_combine_grid), for A/B measurements
_AXES_FOLD = os.environ.get("PYAS_AXES_FOLD", "1") != "0"


# Resident repeat queries: per-store cache of device plans, keyed by the
# query (index of slices/Ellipsis, reduced axes, missing-data values)
_PLAN_CACHE_CAP = 64
_MISS = object()


def _index_key(index):
    """Hashable form of an index made of slices, Ellipsis and 1-D integer
    index lists (the box queries a plan can be replayed for); None
    otherwise."""
    if not isinstance(index, tuple):
        index = (index,)
    out = []
    for x in index:
        if x is Ellipsis:
            out.append(("e",))
        elif isinstance(x, (list, np.ndarray)):
            a = np.asarray(x)
            if a.ndim != 1 or a.dtype.kind not in "iu":
                return None
            out.append(("l",) + tuple(int(v) for v in a))
        elif isinstance(x, slice):
            part = ["s"]
            for v in (x.start, x.stop, x.step):
                if v is None:
                    part.append(None)
                elif isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)):
                    part.append(int(v))
                else:
                    return None
            out.append(tuple(part))
        else:
            return None
    return tuple(out)


def _missing_key(missing):
    key = []
    for m in missing:
        if m is None:
            key.append(None)
        else:
            a = np.asarray(m)
            key.append((a.dtype.str, a.shape, a.tobytes()))
    return tuple(key)


class _CachedQuery:
    """A resident query's device plan, replayed by later identical queries:
    no indexer, no chunk table, no uploads or allocations, only the
    launches, the result copy and the formatting (``active.py:591-630``)."""

    def __init__(self, plan, final_shape, grid=None):
        self.plan = plan
        self.final_shape = final_shape
        self.grid = grid            # None: full reduction; else _grid_partials' record
        self.fmt = {}               # format buffers by result dtype / components
        # one replay at a time: the plan's device buffers (partials, total,
        # tie flags, result buffers) are shared by every replay of this key
        self.lock = threading.Lock()

    def run(self, act):
        with self.lock:
            return self._run(act)

    def _run(self, act):
        ctx = self.plan.ctx
        st = ctx.thread_stream()
        shape = self.final_shape
        if self.grid is None:
            final = act._total(self.plan, st)
            return act._format(final.reshape(shape), shape)
        g = self.grid
        if g["folded"]:
            g["tie"]["fused"] = act._fold(ctx, st, self.plan, g["g"], g["fin"].ptr, g["zs_ok"])
        else:   # records of this replay's method (one size per dtype: the buffer fits every method)
            g["rec"] = engine.method_rec(act._method)
            g["zs1"] = act._reduce_axes_zs(ctx, st, self.plan, g["axes_mask"], g["obuf"].ptr, g["parts"].ptr,
                                           g["rec"], g.get("zs_ok1", False))
            g["zs2"] = act._combine_zs(ctx, st, g["parts"].ptr, g["g"], g["fin"].ptr, g["rec"], g["zs1"])
        act._tie_grid(ctx, st, self.plan, g)
        return act._format_device(ctx, st, g["fin"], g["n_final"], shape, bufs=self.fmt)


def release_resident(variable) -> None:
    """Free the HBM copy that resident-mode ``Active`` queries keep for
    ``variable`` (e.g. after the file changed).  Queries already using the
    copy keep it until they finish; the last one frees it."""
    with _RESIDENT_LOCK:
        store = getattr(variable, "_pyas_resident", None)
        if store is None:
            return
        variable._pyas_resident = None
        store["released"] = True
        free = store["users"] == 0
    if free:
        store["buf"].free()


class _External:
    """A device buffer owned by the caller (attach_resident): never freed here."""

    def __init__(self, ptr, owner):
        self.ptr = int(ptr)
        self.owner = owner          # keeps the caller's allocation alive

    def free(self):
        self.owner = None


def _check_attached(variable, device) -> None:
    """A caller-attached resident copy serves queries on its own device only
    (replacing it would drop the caller's allocation behind their back)."""
    store = getattr(variable, "_pyas_resident", None)
    if store is not None and store["device"] != device and isinstance(store["buf"], _External):
        raise ValueError(f"the variable's resident copy was attached on device {store['device']}, "
                         f"not on this query's device {device} (attach_resident)")


def attach_resident(variable, ptr, device: int = 0, owner=None) -> None:
    """Register chunks already decoded in HBM as ``variable``'s resident copy:
    ``ptr`` holds every chunk of the variable's grid in C order, one slot of
    ``ceil(chunk_bytes / 256) * 256`` bytes each, in the variable's dtype
    and byte order (variables without filters only).  Resident-mode queries on
    ``variable`` then read only HBM, as if an earlier query had loaded every
    chunk (a producer on the GPU handing its output to the reduction without
    a trip through a file).  ``owner`` (e.g. the torch tensor behind ``ptr``)
    is kept alive until :func:`release_resident`."""
    ds = variable
    if ds.filter_pipeline:
        raise NotImplementedError("attach_resident: variables with a filter pipeline")
    if int(ptr) % _ALIGN:
        raise ValueError(f"attach_resident: ptr must be {_ALIGN}-byte aligned (chunk slots of the resident layout)")
    grid = tuple(-(-s // c) for s, c in zip(ds.shape, ds.chunks))
    n_all = int(np.prod(grid))
    with _RESIDENT_LOCK:
        if getattr(ds, "_pyas_resident", None) is not None:
            raise ValueError("the variable already has a resident copy (release_resident first)")
        ds._pyas_resident = {"device": int(device), "buf": _External(ptr, owner),
                             "state": np.full(n_all, _LOADED, dtype=np.int8), "users": 0,
                             "released": False}


def _unhold(store) -> None:
    """A query that used ``store`` has finished (its stream is synchronised)."""
    with _RESIDENT_LOCK:
        store["users"] -= 1
        free = store["users"] == 0 and store["released"]
    if free:
        store["buf"].free()


# read -> inflate pipeline stages of a compressed query (PYAS_INFLATE_GROUPS)
_INFLATE_GROUPS = int(os.environ.get("PYAS_INFLATE_GROUPS", "3"))

# Where Active inflates zlib chunks when device_inflate="auto" (row f3).  One
# pyas_inflate stream is one serial DEFLATE decoder (~135 MB/s, two waves per
# stream), so the device finishes up to ~2048 streams in about one stream's
# time, while the host inflates on its reader threads -- one per pinned
# staging slot in flight, min(threads, 16) -- at zlib's per-core rate and
# takes ceil(n / lanes) stream times: the device wins from about lanes x
# (host rate / device rate) streams.  Measured on MI355X with
# tools/bench_inflate_crossover.py (profiles/r06/crossover/);
# PYAS_INFLATE_CROSSOVER overrides the streams per host lane below which the
# host inflates.
_INFLATE_CROSSOVER = float(os.environ.get("PYAS_INFLATE_CROSSOVER", "10"))
_INGEST_LANES = 16   # pinned staging slots of pyas_read_ranges (ingest.py set_slots)


def inflate_on_device(n_streams: int, threads: int, mode="auto") -> bool:
    """The device/host choice for one query's zlib chunks: ``mode`` True /
    False force it; "auto" inflates on the device from ``_INFLATE_CROSSOVER``
    streams per host inflate lane (PYAS_ACTIVE_INFLATE=device|host overrides
    "auto")."""
    if mode == "auto":
        mode = {"device": True, "host": False}.get(os.environ.get("PYAS_ACTIVE_INFLATE", ""), "auto")
    if mode != "auto":
        return bool(mode)
    lanes = max(1, min(int(threads), _INGEST_LANES))
    return n_streams >= _INFLATE_CROSSOVER * lanes


def _pipeline_groups(sizes, n_groups):
    """Up to ``n_groups`` contiguous index ranges of about equal total size."""
    z = np.asarray(sizes, dtype=np.int64)
    if z.size == 0:
        return []
    cum = np.cumsum(z)
    cuts = np.searchsorted(cum, cum[-1] * np.arange(1, max(1, n_groups)) / max(1, n_groups), side="left") + 1
    edges = np.unique(np.concatenate([[0], np.minimum(cuts, z.size), [z.size]]))
    return [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:]) if b > a]



# PYAS_ZERO_SIGN_FALLBACK=warn: a query whose zero-sign pass the device cannot
# run returns the reduction with the device's sign of a zero min/max and a
# RuntimeWarning, instead of raising (the default keeps NumPy's bytes or fails)
_SIGN_FALLBACK_WARN = os.environ.get("PYAS_ZERO_SIGN_FALLBACK", "") == "warn"


def _sign_fallback(err):
    """A zero-sign pass the device cannot run for this query (e.g. 2^31 or
    more reduced elements per output: its scan keys are 32-bit).  Raises
    ``err`` unless the caller opted in (PYAS_ZERO_SIGN_FALLBACK=warn): the
    reduction itself is complete, but the sign of a zero min/max would be the
    device reduction's rather than NumPy's (storage.py:99-100)."""
    if not _SIGN_FALLBACK_WARN:
        raise err
    warnings.warn(f"the sign of a zero min/max is not NumPy's for this query ({err})",
                  RuntimeWarning, stacklevel=3)

class Active:
    """GPU-backed ``Active`` over one chunked variable."""

    def __new__(cls, *args, **kwargs):
        inst = super().__new__(cls)
        inst._methods = {"min": np.ma.min, "max": np.ma.max, "sum": np.ma.sum, "mean": np.ma.sum}
        return inst

    def __init__(self, dataset, ncvar=None, axis=None, interface_type=None, max_threads: int = 30,
                 storage_options=None, active_storage_url=None, option_disable_chunk_cache=False,
                 *, device: int = 0, device_inflate="auto", group=None, resident: bool = False):
        """``dataset``: a netCDF4/HDF5 file path with ``ncvar`` naming the
        variable (``active.py:185-280``: same signature, checks and errors),
        or a :class:`ChunkedVariable` (the reference accepts a pyfive
        Dataset).  Local files only: ``interface_type`` "s3"/"https" and
        ``storage_options`` (remote object stores) are not served here."""
        if interface_type not in (None, "", "posix", "ActivePosix") or storage_options is not None:
            raise NotImplementedError(
                f"interface_type={interface_type!r}: remote object stores are outside this backend; "
                "point Reductionist clients at pyactivestorage_amd.reductionist_server instead")
        self.active_storage_url = active_storage_url
        self.option_disable_chunk_cache = bool(option_disable_chunk_cache)
        if dataset is None:
            raise ValueError(f"Must use a valid file name or variable object for dataset. Got {dataset!r}")
        if isinstance(dataset, (str, os.PathLike)):
            path = os.fspath(dataset)
            if not os.path.isfile(path):
                raise ValueError(f"Must use existing file for uri. {path} not found")
            if ncvar is None:
                raise ValueError("Must set a netCDF variable name to slice")
            from .hdf5 import open_variable
            variable = open_variable(path, ncvar)
        elif isinstance(dataset, ChunkedVariable):
            variable = dataset
        else:
            raise TypeError(f"Variable object dataset can only be a ChunkedVariable. Got {dataset!r}")
        self.uri = dataset
        self.ncvar = ncvar
        self.ds = variable
        if axis is not None:
            axis = (axis,) if isinstance(axis, int) else tuple(axis)
        self._axis = axis
        self._components = False
        self._method = None
        self._max_threads = int(max_threads)
        self.device = device
        # f3: zlib chunks inflate on the GPU (True), on the host reader threads
        # straight into the pinned ring (False), or whichever is faster for the
        # query's stream count ("auto", inflate_on_device)
        if device_inflate not in (True, False, "auto"):
            raise ValueError(f"device_inflate must be True, False or 'auto'. Got {device_inflate!r}")
        self.device_inflate = device_inflate
        # row (e): a torch.distributed process group (one process per GPU).
        # Each rank reads and reduces a contiguous range of the query's chunks
        # from its own GPU; one all-gather of the per-rank partial grids and a
        # fixed rank-order device combine give every rank the same result.
        self.group = group
        # keep the variable's decoded chunks in HBM across queries (288 GB per
        # MI355X): later queries read only chunks not loaded yet
        self.resident = bool(resident)
        self.missing = None
        self.data_read = 0
        self._held = threading.local()

    # -- API mirrored from active.py:355-418 ------------------------------
    @property
    def components(self):
        return self._components

    @components.setter
    def components(self, value):
        self._components = bool(value)

    @property
    def method(self):
        return self._methods.get(self._method)

    @method.setter
    def method(self, value):
        if value is not None and value not in self._methods:
            raise ValueError(f"Bad 'method': {value}. Choose from min/max/mean/sum.")
        self._method = value

    def mean(self, axis=None):
        self._method = "mean"
        if axis is not None:
            self._axis = axis
        return self

    def min(self, axis=None):
        self._method = "min"
        if axis is not None:
            self._axis = axis
        return self

    def max(self, axis=None):
        self._method = "max"
        if axis is not None:
            self._axis = axis
        return self

    # -- query -------------------------------------------------------------
    def __getitem__(self, index):
        self.missing = get_missing_attributes(self.ds.attrs)
        self.data_read = 0
        held = self._held.stores = []    # resident stores this query uses (this thread)
        try:
            return self._get_selection(index)
        finally:
            self._method = None          # active.py:633
            for store in held:
                _unhold(store)
            self._held.stores = []

    def _get_selection(self, index):
        ds = self.ds
        if self._axis is None:
            self._axis = tuple(range(ds.ndim))
        elif isinstance(self._axis, int):
            self._axis = (self._axis,)
        cache_key = None
        if self.resident and self.group is None and self._method is not None:
            ikey = _index_key(index)
            if ikey is not None:
                cache_key = (ikey, self._norm_axes(), _missing_key(self.missing))
                hit = self._cached_query(cache_key)
                if hit is not _MISS:
                    return hit
        compressor, filters = (None, None) if not ds.filter_pipeline else \
            decode_filters(ds.filter_pipeline, ds.dtype.itemsize, ds.name)
        indexer = OrthogonalIndexer(index, ds.shape, ds.chunks)
        if self.components and self._method is None:       # active.py:483-485
            raise ValueError("Setting components to True for None statistical method.")
        if self._method is None:
            return self._select(indexer, compressor, filters)
        for i, d in enumerate(indexer.dim_indexers):        # active.py:489-500
            if d.kind == "int":
                raise IndexError("Can't do an active reduction when the index for "
                                 f"axis {i!r} drops the axis.")
        return self._reduce(indexer, compressor, filters, self._norm_axes(), cache_key)

    def _norm_axes(self):
        """The reduced axes, sorted and non-negative (active.py:505-510)."""
        ndim = self.ds.ndim
        axes = []
        for i in self._axis:
            if not -ndim <= i < ndim:
                raise ValueError(f"Can't do an active reduction for an out-of-range axis: {i!r}")
            axes.append(i % ndim)
        if len(set(axes)) != len(axes):
            raise ValueError("duplicate value in 'axis'")
        return tuple(sorted(axes))

    def _cached_query(self, key):
        """Replay a cached plan of this resident variable (every chunk of the
        query is still in its slot), or _MISS."""
        store = getattr(self.ds, "_pyas_resident", None)
        if store is None or store["device"] != self.device:
            return _MISS
        with _RESIDENT_LOCK:
            entry = store.get("plans", {}).get(key)
            if entry is None or store["released"]:
                return _MISS
            store["users"] += 1
        self._held.stores.append(store)
        return entry.run(self)

    def _remember(self, key, entry):
        store = getattr(self.ds, "_pyas_resident", None)
        if key is None or store is None or entry.plan.batch.data != store["buf"].ptr:
            return
        with _RESIDENT_LOCK:
            plans = store.setdefault("plans", {})
            if len(plans) >= _PLAN_CACHE_CAP:
                plans.pop(next(iter(plans)))
            plans[key] = entry

    # -- host ingest -------------------------------------------------------
    def _ingest(self, coords, compressor, filters):
        """Device buffer + per-chunk offsets of every touched chunk (decoded,
        still byte-shuffled when the shuffle is fused into the kernels).
        ``coords``: chunk coordinate tuples, or an int64 array (n, ndim)."""
        if self.resident:
            got = self._ingest_resident(coords, compressor, filters)
            if got is not None:
                return got
        if isinstance(coords, np.ndarray):
            coords = [tuple(c) for c in coords.tolist()]
        return self._ingest_fresh(coords, compressor, filters)

    def _ingest_resident(self, coords, compressor, filters):
        """Resident mode: the variable's decoded chunks stay in HBM (one slot
        per chunk of the variable's grid, allocated on first use), so a query
        reads from the file only the chunks no earlier query loaded.  None
        when the filter pipeline needs a standalone device pass."""
        ds = self.ds
        shuffles = _shuffle_sizes(filters)
        if shuffles and shuffles[-1] == ds.dtype.itemsize:
            shuffles.pop()
        if any(es > 1 for es in shuffles):
            return None
        nbytes = int(np.prod(ds.chunks)) * ds.dtype.itemsize
        stride = -(-nbytes // _ALIGN) * _ALIGN
        grid = tuple(-(-s // c) for s, c in zip(ds.shape, ds.chunks))
        _check_attached(ds, self.device)
        ctx = get_context(self.device)
        with _RESIDENT_LOCK:
            store = getattr(ds, "_pyas_resident", None)
            _check_attached(ds, self.device)
            if store is None or store["device"] != self.device:
                n_all = int(np.prod(grid))
                store = {"device": self.device, "buf": DeviceBuffer(ctx, max(n_all, 1) * stride),
                         "state": np.zeros(n_all, dtype=np.int8), "users": 0, "released": False}
                ds._pyas_resident = store
            store["users"] += 1
        held = getattr(self._held, "stores", None)
        if held is None:
            held = self._held.stores = []
        held.append(store)
        c = np.asarray(coords, dtype=np.int64).reshape(len(coords), len(grid))
        slots = np.ravel_multi_index(c.T, grid) if len(coords) else np.zeros(0, dtype=np.int64)
        fused = self._fused_shuffle(filters)
        st = ctx.thread_stream()
        while True:
            # claim the empty slots; slots another query is loading are waited for
            with _RESIDENT_LOCK:
                state = store["state"]
                todo = np.nonzero(state[slots] == _EMPTY)[0]
                state[slots[todo]] = _LOADING
            try:
                st = self._load_slots(ctx, store, c[todo], slots[todo], stride, nbytes, compressor,
                                      filters, fused)
            except BaseException:
                with _RESIDENT_CV:
                    store["state"][slots[todo]] = _EMPTY
                    _RESIDENT_CV.notify_all()
                raise
            with _RESIDENT_CV:
                store["state"][slots[todo]] = _LOADED
                _RESIDENT_CV.notify_all()
                while (store["state"][slots] == _LOADING).any():
                    _RESIDENT_CV.wait()
                if (store["state"][slots] == _LOADED).all():
                    break
                # a loader failed: its slots are empty again, claim them
        return ctx, st, store["buf"], slots.astype(np.int64) * stride, 0 if fused in (2, 4, 8) else fused

    def _load_slots(self, ctx, store, coords, slots, stride, nbytes, compressor, filters, fused):
        """Read + decode chunks ``coords`` into resident ``slots``; returns
        the stream, synchronised (other queries read the slots once marked)."""
        st = ctx.thread_stream()
        if not len(slots):
            return st
        todo_coords = [tuple(x) for x in coords.tolist()]
        if fused in (2, 4, 8):
            # the store keeps chunks un-shuffled (one batched pass as they
            # arrive), so every later query takes the unshuffled kernels
            # (dense partial-axis layouts and the in-kernel layer fold)
            _, st, tmp, toffs, _ = self._ingest_fresh(todo_coords, compressor, filters)
            offs = np.concatenate([toffs, slots * stride]).astype(np.int64)
            meta = DeviceBuffer(ctx, offs.nbytes)
            ctx.h2d(meta.ptr, offs, st)
            engine.unshuffle_chunks(ctx, tmp.ptr, meta.ptr, store["buf"].ptr, meta.ptr + 8 * len(slots),
                                    len(slots), nbytes, fused, st)
            ctx.synchronize(st)   # tmp and meta are freed on return
        else:
            _, st, _, _, _ = self._ingest_fresh(todo_coords, compressor, filters,
                                                dst=store["buf"], dst_offsets=slots * stride)
            ctx.synchronize(st)
        return st

    def _ingest_fresh(self, coords, compressor, filters, dst=None, dst_offsets=None):
        """Read + inflate every touched chunk into one device buffer (``dst``
        at ``dst_offsets`` when given)."""
        ds = self.ds
        nbytes = int(np.prod(ds.chunks)) * ds.dtype.itemsize

        zlib_chunks = is_zlib(compressor)
        device_inflate = zlib_chunks and inflate_on_device(len(coords), self._max_threads, self.device_inflate)
        ctx = get_context(self.device)
        st = ctx.thread_stream()
        stride = -(-nbytes // _ALIGN) * _ALIGN
        infos = [ds.chunk_info(c) for c in coords]
        n = len(infos)
        doffs = (np.arange(n, dtype=np.int64) * stride if dst_offsets is None
                 else np.ascontiguousarray(dst_offsets, dtype=np.int64))
        if n == 0:
            buf = dst if dst is not None else DeviceBuffer(ctx, stride)
            return ctx, st, buf, doffs, self._fused_shuffle(filters)
        native_io = ds.reader is None and ds.filename is not None and (zlib_chunks or compressor is None)
        if native_io:
            # f2: native pread ring -> pinned slots -> H2D, no Python per chunk
            foff = np.array([o for o, _ in infos], dtype=np.int64)
            fsize = np.array([z for _, z in infos], dtype=np.int64)
            self.data_read += int(fsize.sum())
            if device_inflate:
                # f2+f3 pipeline: the compressed bytes arrive in groups on a
                # copy stream; each group is inflated on its own stream as soon
                # as its copies land (inflate waves of every group can be
                # resident together: one stream per wave, so concurrency is
                # what buys inflate throughput), while the host reads on
                # compressed streams back to back (the inflater reads any
                # alignment), so file-contiguous chunks stay one H2D copy per
                # staging slot instead of one per chunk
                soffs = np.concatenate([[0], np.cumsum(fsize)[:-1]]).astype(np.int64)
                src = DeviceBuffer(ctx, int(fsize.sum()) + 16)
                buf = dst if dst is not None else DeviceBuffer(ctx, max(n, 1) * stride)
                copy_st = ctx.thread_aux_stream(0)
                ctx.stream_wait(copy_st, st)      # order after prior work on st
                batches = []
                # one launch per ~2048 streams: below that a launch inflates
                # every stream at once (a stream's time is the latency of one
                # serial decoder), so splitting the read/inflate pipeline into
                # launches would only queue them one after another
                groups = _pipeline_groups(fsize, max(1, min(_INFLATE_GROUPS, -(-n // 2048))))
                for g, (lo, hi) in enumerate(groups):
                    read_ranges(ctx, ds.filename, foff[lo:hi], fsize[lo:hi], src.ptr, soffs[lo:hi],
                                copy_st, self._max_threads)
                    inf_st = ctx.thread_aux_stream(1 + g)
                    ctx.stream_wait(inf_st, copy_st)
                    ib = InflateBatch(ctx, soffs[lo:hi], fsize[lo:hi], doffs[lo:hi],
                                      np.full(hi - lo, nbytes, dtype=np.int64))
                    ib.launch(src.ptr, buf.ptr, inf_st)
                    batches.append((lo, ib, inf_st))
                for lo, ib, inf_st in batches:
                    ib.check(inf_st, base=lo)
                    ctx.stream_wait(st, inf_st)
                del src
            elif zlib_chunks:
                # f3 on the host: the reader threads inflate each chunk straight
                # into its pinned staging slot (pyas_read_ranges_zlib), the
                # inflated bytes go H2D
                buf = dst if dst is not None else DeviceBuffer(ctx, max(n, 1) * stride)
                read_ranges_zlib(ctx, ds.filename, foff, fsize, buf.ptr, doffs, nbytes, st, self._max_threads,
                                 reshape=(ds.dtype.itemsize, ds.chunks))
            else:
                bad = np.nonzero(fsize != nbytes)[0]
                if bad.size:   # storage.py:57-62 reshape of a wrongly sized chunk
                    raise ValueError(f"cannot reshape array of size {int(fsize[bad[0]]) // ds.dtype.itemsize} "
                                     f"into shape {ds.chunks}")
                buf = dst if dst is not None else DeviceBuffer(ctx, max(n, 1) * stride)
                read_ranges(ctx, ds.filename, foff, fsize, buf.ptr, doffs, st, self._max_threads)
        else:
            def fetch(info):
                off, size = info
                raw = ds.read(off, size)
                return off, size, (raw if device_inflate else _decompress(raw, compressor))

            with concurrent.futures.ThreadPoolExecutor(max_workers=self._max_threads) as ex:
                blobs = list(ex.map(fetch, infos))
            if device_inflate:
                # f3: one upload of the deflated bytes, one inflate launch into the
                # chunk-major slots the reduce reads (raises like zlib.decompress)
                host, soffs, ssizes = pack_streams([b for _, _, b in blobs])
                self.data_read += int(ssizes.sum())
                src = DeviceBuffer(ctx, host.nbytes)
                ctx.h2d(src.ptr, host, st)
                buf = dst if dst is not None else DeviceBuffer(ctx, max(n, 1) * stride)
                ib = InflateBatch(ctx, soffs, ssizes, doffs, np.full(n, nbytes, dtype=np.int64))
                ib.launch(src.ptr, buf.ptr, st)
                ib.check(st)
                del src
            else:
                host = np.zeros(max(n, 1) * stride, dtype=np.uint8)
                for i, (_, size, b) in enumerate(blobs):
                    a = np.frombuffer(memoryview(b), dtype=np.uint8)
                    if a.size != nbytes:
                        raise ValueError(f"cannot reshape array of size {a.size // ds.dtype.itemsize} "
                                         f"into shape {ds.chunks}")
                    host[i * stride: i * stride + nbytes] = a
                    self.data_read += size
                if dst is None:
                    buf = DeviceBuffer(ctx, host.nbytes)
                    ctx.h2d(buf.ptr, host, st)
                else:
                    buf = dst
                    for i in range(n):
                        ctx.h2d(buf.ptr + int(doffs[i]), host[i * stride: (i + 1) * stride], st)
        shuffles = _shuffle_sizes(filters)
        fused = self._fused_shuffle(filters)
        if shuffles and shuffles[-1] == ds.dtype.itemsize:
            shuffles.pop()
        for es in shuffles:   # non-itemsize shuffles: standalone device pass per chunk
            if es > 1:
                assert dst is None   # resident mode keeps such pipelines out
                tmp = DeviceBuffer(ctx, buf.nbytes)
                for i in range(n):
                    engine.unshuffle(ctx, buf.ptr + i * stride, tmp.ptr + i * stride, nbytes, es, st)
                buf = tmp
        return ctx, st, buf, doffs, fused

    def _fused_shuffle(self, filters):
        """Element size of the shuffle the kernels undo on load (0: none)."""
        shuffles = _shuffle_sizes(filters)
        es = self.ds.dtype.itemsize
        return es if shuffles and shuffles[-1] == es and es > 1 else 0

    @staticmethod
    def _chunk_sel(projs):
        dims = []
        for p in projs:
            s = p.chunk_sel
            if isinstance(s, slice):
                cnt = len(p.out_pos)
                dims.append(selection.DimSel(s.start if cnt else 0, s.step, cnt, False))
            elif isinstance(s, np.ndarray):
                dims.append(selection.DimSel(0, 0, int(s.size), False, s.astype(np.int64)))
            else:
                dims.append(selection.DimSel(int(s), 1, 1, True))
        shape = tuple(d.count for d in dims if not d.dropped)
        kept = tuple(i for i, d in enumerate(dims) if not d.dropped)
        return selection.ChunkSel(dims, shape, kept)

    # -- reductions ---------------------------------------------------------
    def _box_plan(self, indexer):
        """Vectorised plan of an orthogonal selection of slices and index
        arrays: the touched chunks are the C-ordered product of per-dim
        projections (active.py:451-471), so the ABI selection table, index
        pool and chunk coordinates follow from per-dim entries by
        broadcasting, with no per-chunk Python objects.  Returns
        ``(dims, coords, table, pool)`` or None (integer-dropped dims, or
        vector fill/missing values whose masks need per-chunk selections)."""
        if any(d.kind == "int" for d in indexer.dim_indexers):
            return None
        if any(m is not None and np.size(m) != 1 for m in self.missing):
            return None
        dims = [list(d) for d in indexer.dim_indexers]
        nd = len(dims)
        n_coords = [len(p) for p in dims]
        ent, pool_parts, pos = [], [], 0
        for projs in dims:
            e = np.zeros((len(projs), 3), dtype=np.int32)
            for a, p in enumerate(projs):
                sl = p.chunk_sel
                if isinstance(sl, slice):
                    cnt = len(p.out_pos)
                    e[a] = (sl.start if cnt else 0, sl.step, cnt)
                else:
                    e[a] = (pos, 0, sl.size)
                    pool_parts.append(np.asarray(sl, dtype=np.int32))
                    pos += sl.size
            ent.append(e)
        n = int(np.prod(n_coords))
        idx = np.indices(n_coords).reshape(nd, n)
        table = np.zeros((n, _lib.MAX_DIMS, 3), dtype=np.int32)
        table[:, :, 1] = 1
        table[:, :, 2] = 1
        coords = np.zeros((n, nd), dtype=np.int64)
        for d in range(nd):
            table[:, d, :] = ent[d][idx[d]]
            coords[:, d] = np.array([p.chunk_ix for p in dims[d]], dtype=np.int64)[idx[d]]
        pool = np.concatenate(pool_parts) if pool_parts else np.zeros(1, dtype=np.int32)
        return dims, coords, table, pool

    def _reduce(self, indexer, compressor, filters, axes, cache_key=None):
        box = self._box_plan(indexer)
        if box is None:
            if self.group is not None:
                raise NotImplementedError("a distributed Active query needs slices/index lists on every "
                                          "dimension and scalar missing-data attributes")
            return self._reduce_general(indexer, compressor, filters, axes)
        ds = self.ds
        dt = ds.dtype
        dims, coords, table, pool = box
        final_shape = tuple(1 if i in axes else n for i, n in enumerate(indexer.shape))
        n_final = int(np.prod(final_shape))
        pdt = engine.partial_dtype(dt)
        n = len(coords)
        lo, hi = 0, n
        if self.group is not None:   # this rank's contiguous chunk range
            import torch.distributed as dist
            from .distributed import shard_ranges
            weights = np.prod(table[:, :ds.ndim, 2].astype(np.int64), axis=1)
            lo, hi = shard_ranges(weights, dist.get_world_size(self.group))[dist.get_rank(self.group)]
        keys = [] if self.group is not None else None
        if hi > lo:
            ctx, st, buf, offsets, fused = self._ingest(coords[lo:hi], compressor, filters)
            sub = table[lo:hi]
            full = _all_full(sub, ds.chunks)   # whole chunks: no table, lean/dense kernels
            plan = ReductionPlan(ctx, dt, ds.chunks, buf.ptr, offsets, shuffle=fused,
                                 sel_table=None if full else sub, index_pool=None if full else pool,
                                 missing=self.missing, round_to_var=True, stream=st)
            cacheable = cache_key is not None and self.resident and self.group is None
            if len(axes) == ds.ndim:
                final = self._total(plan, st, layer_base=lo, n_layers=n, keys=keys)
                if cacheable:
                    self._remember(cache_key, _CachedQuery(plan, final_shape))
            else:
                grid = self._grid_from_dims(dims, axes, final_shape)
                if self.group is None:   # one process: format on the device
                    rec = {} if cacheable else None
                    out = self._grid_partials(ctx, st, plan, grid, axes, final_shape, lo, hi,
                                              formatted=True, rec=rec)
                    if cacheable:
                        self._remember(cache_key, _CachedQuery(plan, final_shape, rec))
                    return out
                final = self._grid_partials(ctx, st, plan, grid, axes, final_shape, lo, hi, keys=keys)
        else:
            final = np.zeros(n_final, dtype=pdt)   # count 0: neutral in every combine
        if self.group is not None:
            if not keys:   # no chunks here, or no zero-sign work: neutral keys
                keys = [np.concatenate([np.zeros(n_final, np.uint64), np.full(n_final, ~np.uint64(0))])]
            lr = n if len(axes) == ds.ndim else \
                zerosign.grid_lr([len(dims[d]) if d in axes else final_shape[d] for d in range(ds.ndim)],
                                 set(axes))
            final = self._exchange(final, keys[0], lr)
        return self._format(final.reshape(final_shape), final_shape)

    def _tie_which(self) -> int:
        """1 / 2 when the query's min / max of a float variable must give
        NumPy's sign of a zero extreme (pyas_tie_*), else 0."""
        if self.ds.dtype.kind != "f":
            return 0
        return {"min": 1, "max": 2}.get(self._method, 0)

    def _total(self, plan, st, layer_base=0, n_layers=None, keys=None):
        """Full reduction of the plan's chunks: the combined partial.  For
        min/max of a float variable the chunk partials are kept so that a
        zero extreme gets NumPy's sign: per chunk over its elements
        (storage.py:99-100, pyas_tie_chunks), then over the per-chunk values
        in the `out` array's C order (active.py:594, pyas_tie_segments);
        level 1 scans only the two chunks level 2 can pick
        (pyas_tie_chunks_total).
        Under a group the plan holds this rank's chunks, the first at
        position ``layer_base`` of the ``n_layers`` in the query, and the
        level-2 keys go to ``keys`` (a host list) for pyas_tie_finalize
        after the exchange."""
        which = self._tie_which()
        plan.launch(st, chunk_partials=bool(which))
        if which:
            ctx, dt = plan.ctx, self.ds.dtype
            n_all = plan.n_chunks if n_layers is None else int(n_layers)
            # level 1 only on the chunks the level-2 keys can pick (positions
            # decide which zero wins; the two candidates' signs are then exact)
            try:
                engine.tie_chunks_total(ctx, plan.batch, plan.mask_up.struct, plan.tie_geom(), which,
                                        plan.chunk_partials.ptr, int(layer_base), max(n_all, 1), st)
            except NotImplementedError as e:
                if keys is not None:
                    raise
                _sign_fallback(e)
                return plan.read_total(st)
            kbuf = None
            if keys is not None:
                kbuf = DeviceBuffer(ctx, 16)
                engine.tie_keys_reset(ctx, kbuf.ptr, 1, st)
            # `out` is one coordinate per chunk and every dim reduced: one call of n_all
            engine.tie_segments(ctx, dt, plan.chunk_partials.ptr, None, None, 1, plan.n_chunks, int(layer_base),
                                max(n_all, 1), which, plan.total.ptr, kbuf.ptr if kbuf else None, st)
            if kbuf is not None:
                host = np.zeros(2, dtype=np.uint64)
                ctx.d2h(host, kbuf.ptr, st)
                ctx.synchronize(st)
                keys.append(host)
        return plan.read_total(st)

    def _reduce_axes_zs(self, ctx, st, plan, axes_mask, obuf_ptr, parts_ptr, prec, zs_ok1) -> bool:
        """pyas_reduce_axes_ex into records; with PYAS_REC_ZERO_SIGN when
        the query is a min/max whose level-1 zero sign the walk can key
        (``zs_ok1``).  Returns whether it did (then pyas_tie_chunks is not
        needed)."""
        if zs_ok1 and self._tie_which() and prec in (_lib.REC_MIN, _lib.REC_MAX):
            try:
                engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, axes_mask, obuf_ptr, parts_ptr, st,
                                   rec=prec | _lib.REC_ZERO_SIGN)
                return True
            except NotImplementedError:
                pass   # another layout: the scan pass keys the sign
        # every chunk whole or a box the dense launch takes: no generic walk
        # every chunk whole or a box the dense launch takes: no generic walk;
        # no chunk of the dense launch's: no dense launch
        dense = _lib.REC_DENSE_ONLY if prec and plan.dense_boxes() else \
            _lib.REC_GENERIC_ONLY if prec and plan.no_dense_boxes() else 0
        engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, axes_mask, obuf_ptr, parts_ptr, st, rec=prec | dense)
        return False

    def _tie_grid(self, ctx, st, plan, rec, keys_ptr=None):
        """NumPy's sign of the zero min/max outputs of a partial-axis box
        query (``rec``: _grid_partials' record): per chunk output
        (storage.py:99-100), then over the chunk layers of the `out` array
        (active.py:594)."""
        which = self._tie_which()
        if not which:
            return
        t = rec["tie"]
        if t.get("fused"):   # the fold wrote NumPy's sign itself (elementwise at both levels)
            return
        dt = self.ds.dtype
        geom = plan.tie_geom()
        if rec["folded"]:   # no per-chunk partials: per chunk output flags
            if t.get("flags") is None:
                t["flags"] = DeviceBuffer(ctx, max(t["n_parts"], 1))
            engine.tie_chunk_flags(ctx, plan.batch, plan.mask_up.struct, geom, rec["axes_mask"], which,
                                   rec["obuf"].ptr, rec["fin"].ptr, rec["n_final"], t["flags"].ptr, st)
            engine.tie_grid(ctx, dt, rec["g"], None, t["flags"].ptr, t["lr"], which, rec["fin"].ptr, keys_ptr, st)
        else:   # per-chunk partials: compact records of the method (pyas_reduce_axes_ex)
            pw = which | (_lib.TIE_REC if rec.get("rec") else 0)
            if rec.get("zs2") and keys_ptr is None:   # walk and combine keyed both levels
                return
            if rec.get("zs1"):   # the walk keyed level 1 itself: only the `out` level
                engine.tie_grid(ctx, dt, rec["g"], rec["parts"].ptr, None, t["lr"], pw, rec["fin"].ptr, keys_ptr, st)
                return
            try:
                engine.tie_chunks(ctx, plan.batch, plan.mask_up.struct, geom, rec["axes_mask"], pw,
                                  rec["obuf"].ptr, rec["parts"].ptr, st)
            except NotImplementedError as e:
                if keys_ptr is not None:
                    raise
                _sign_fallback(e)
                return
            engine.tie_grid(ctx, dt, rec["g"], rec["parts"].ptr, None, t["lr"], pw, rec["fin"].ptr, keys_ptr,
                            st)

    def _exchange(self, final, keys=None, lr=1):
        """All-gather the per-rank partial grids (RCCL for an nccl group,
        else over the group's CPU backend) and fold them in rank order on
        the device (pyas_combine_segments).  ``keys``: this rank's zero-sign
        keys (2 x n uint64), gathered in the same collective and combined
        by pyas_tie_finalize, so a zero min/max carries NumPy's sign over
        the whole `out` array (active.py:594).  Every rank gets the result."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(self.group)
        which = self._tie_which() if keys is not None else 0
        n = final.size
        ctx = get_context(self.device)
        st = ctx.thread_stream()
        if world == 1 and not which:
            return final
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        blob = np.ascontiguousarray(final).view(np.uint8).reshape(-1)
        if which:
            blob = np.concatenate([blob, np.ascontiguousarray(keys, dtype=np.uint64).view(np.uint8)])
        t = torch.from_numpy(blob.copy()).to(dev)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=self.group)
        host = [p.cpu().numpy() for p in parts]
        gathered = np.concatenate([h[:final.nbytes] for h in host]).view(final.dtype)
        gkeys = np.concatenate([h[final.nbytes:] for h in host]).view(np.uint64) if which else None
        index = (np.arange(world, dtype=np.int64)[None, :] * n
                 + np.arange(n, dtype=np.int64)[:, None]).reshape(-1)
        seg = np.arange(n + 1, dtype=np.int64) * world
        gbuf = DeviceBuffer(ctx, gathered.nbytes)
        ctx.h2d(gbuf.ptr, gathered, st)
        meta = np.concatenate([index, seg])
        mbuf = DeviceBuffer(ctx, meta.nbytes)
        ctx.h2d(mbuf.ptr, meta, st)
        fin = DeviceBuffer(ctx, max(n, 1) * _lib.PARTIAL_NBYTES)
        engine.combine_segments(ctx, self.ds.dtype, gbuf.ptr, mbuf.ptr, mbuf.ptr + 8 * index.size, n,
                                fin.ptr, False, st)
        if which:
            kb = DeviceBuffer(ctx, gkeys.nbytes)
            ctx.h2d(kb.ptr, gkeys, st)
            engine.tie_finalize(ctx, self.ds.dtype, kb.ptr, n, world, lr, which, fin.ptr, st)
        out = np.zeros(n, dtype=final.dtype)
        ctx.d2h(out, fin.ptr, st)
        ctx.synchronize(st)
        return out

    def _grid_combine(self, ctx, st, plan, grid, axes, final_shape):
        """Partial axes over a box query, every chunk local."""
        return self._grid_partials(ctx, st, plan, grid, axes, final_shape, 0, plan.n_chunks,
                                   formatted=True)

    def _grid_partials(self, ctx, st, plan, grid, axes, final_shape, lo, hi, formatted=False, rec=None,
                       keys=None):
        """Per-chunk partial arrays of chunks [lo, hi) of the box query
        (pyas_reduce_axes over ``plan``), then pyas_combine_grid into the
        final grid; chunks outside [lo, hi) read a zeroed (count 0, neutral)
        partial region.  ``formatted``: return the formatted result
        (``_format_device``) instead of the host partials.  ``rec``: filled
        with what a replay of this query needs (_CachedQuery).  ``keys``
        (group queries): a host list that receives this rank's zero-sign
        keys of every output (pyas_tie_grid), for pyas_tie_finalize."""
        ds = self.ds
        dt = ds.dtype
        n_final = int(np.prod(final_shape))
        axes_mask = 0
        for a in axes:
            axes_mask |= 1 << a
        out_off, tables = grid
        n_all = out_off.size
        n_parts_all = int(tables["n_parts"])
        end = np.append(out_off, n_parts_all)
        base, top = int(end[lo]), int(end[hi])
        neutral = 0
        if lo > 0 or hi < n_all:
            neutral = int(np.diff(end).max())
        mine = out_off[lo:hi] - base
        all_off = np.full(n_all, top - base, dtype=np.int64)   # the neutral region
        all_off[lo:hi] = mine
        obuf = DeviceBuffer(ctx, mine.nbytes)
        ctx.h2d(obuf.ptr, mine, st)
        abuf = DeviceBuffer(ctx, all_off.nbytes)
        ctx.h2d(abuf.ptr, all_off, st)
        tbuf = DeviceBuffer(ctx, max(tables["blob"].nbytes, 16))
        ctx.h2d(tbuf.ptr, tables["blob"], st)
        g = _lib.Grid()
        g.ndim = ds.ndim
        g.axes_mask = axes_mask
        for d in range(ds.ndim):
            g.n_coords[d] = tables["n_coords"][d]
            g.out_extent[d] = final_shape[d] if d not in axes else 1
            if d not in axes:
                g.pos_coord[d] = tbuf.ptr + 4 * tables["pos_coord"][d]
                g.pos_local[d] = tbuf.ptr + 4 * tables["pos_local"][d]
                g.coord_count[d] = tbuf.ptr + 4 * tables["coord_count"][d]
        g.chunk_out_offsets = abuf.ptr
        fin = DeviceBuffer(ctx, max(n_final, 1) * _lib.PARTIAL_NBYTES)
        folded = fused = False
        zs_ok = self._fold_sign_ok(axes)
        if (_AXES_FOLD and lo == 0 and hi == n_all and not plan.batch.sel
                and self._whole_chunk_grid(tables, final_shape, axes)):
            try:   # one launch: chunk layers folded inside the reduction kernel
                fused = self._fold(ctx, st, plan, g, fin.ptr, zs_ok)
                folded = True
            except NotImplementedError:
                pass   # geometry without the dense column or LDS row layout: two steps
        parts = None
        prec = 0
        if not folded:
            # per-chunk outputs as compact records of the method (storage.py:98-100
            # per chunk, the sum rounded as active.py:512 stores it): 8 B per
            # output for <= 4-byte dtypes instead of the 32-B partial
            prec = engine.method_rec(self._method)
            rb = _lib.rec_nbytes(dt.itemsize, prec)
            n_parts = top - base
            parts = DeviceBuffer(ctx, max(n_parts + neutral, 1) * rb)
            if neutral:   # zero records: count 0, neutral in the combine
                zeros = np.zeros(neutral * rb, dtype=np.uint8)
                ctx.h2d(parts.ptr + n_parts * rb, zeros, st)
            # level 1 of NumPy's zero sign keyed by the per-chunk walk itself
            # where it can (PYAS_REC_ZERO_SIGN), else pyas_tie_chunks below
            zs_ok1 = zs_ok and plan.dense_boxes()
        ext = [tables["n_coords"][d] if d in axes else final_shape[d] for d in range(ds.ndim)]
        lr = zerosign.grid_lr(ext, set(axes))
        zs2 = False
        if not folded:
            zs1 = self._reduce_axes_zs(ctx, st, plan, axes_mask, obuf.ptr, parts.ptr, prec, zs_ok1)
            # level 2 in the combine where the `out` calls are elementwise
            # (group queries key it across ranks: pyas_tie_grid below)
            zs2 = self._combine_zs(ctx, st, parts.ptr, g, fin.ptr, prec, zs1 and keys is None)
        r = rec if rec is not None else {}
        if folded:
            zs_ok1 = zs1 = False
        r.update(folded=folded, g=g, fin=fin, obuf=obuf, abuf=abuf, tbuf=tbuf, parts=parts, rec=prec,
                 axes_mask=axes_mask, n_final=n_final, zs_ok=zs_ok, zs_ok1=zs_ok1, zs1=zs1, zs2=zs2,
                 tie={"lr": lr, "n_parts": n_parts_all, "flags": None, "fused": fused})
        if keys is not None and self._tie_which():
            kbuf = DeviceBuffer(ctx, max(n_final, 1) * 16)
            engine.tie_keys_reset(ctx, kbuf.ptr, n_final, st)
            self._tie_grid(ctx, st, plan, r, kbuf.ptr)
            host = np.zeros(2 * n_final, dtype=np.uint64)
            ctx.d2h(host, kbuf.ptr, st)
            ctx.synchronize(st)
            keys.append(host)
        else:
            self._tie_grid(ctx, st, plan, r)
        if formatted:
            return self._format_device(ctx, st, fin, n_final, final_shape)
        final = np.zeros(n_final, dtype=engine.partial_dtype(dt))
        ctx.d2h(final, fin.ptr, st)
        ctx.synchronize(st)
        return final

    def _combine_zs(self, ctx, st, parts_ptr, g, fin_ptr, prec, keyed) -> bool:
        """pyas_combine_grid of the per-chunk records; ``keyed`` (level 1
        keyed by the walk): level 2 of NumPy's zero sign keyed in the same
        launch, for `out` calls of any length.  Returns whether it was."""
        dt = self.ds.dtype
        which = self._tie_which() if keyed else 0
        if which:
            try:
                engine.combine_grid(ctx, dt, parts_ptr, g, fin_ptr, True, st, rec=prec, zero_sign=which)
                return True
            except NotImplementedError:
                pass
        engine.combine_grid(ctx, dt, parts_ptr, g, fin_ptr, True, st, rec=prec)
        return False

    def _fold_sign_ok(self, axes) -> bool:
        """Whether the fold may fuse NumPy's zero sign of this partial-axis
        query (PYAS_FOLD_ZERO_SIGN_*): a float variable with C-ordered chunks
        (storage.py:99-100 then reduces each chunk in the memory order the
        kernels assume) and this host's NumPy rule known.  The library
        refuses (ENOTSUP) the geometries its fold kernels cannot key."""
        ds = self.ds
        if ds.dtype.kind != "f" or getattr(ds, "order", "C") != "C":
            return False
        ctx = get_context(self.device)
        return bool(getattr(ctx, "tie_signs_exact", {}).get("f4" if ds.dtype.itemsize == 4 else "f8"))

    def _fold(self, ctx, st, plan, g, fin_ptr, zs_ok) -> bool:
        """pyas_reduce_axes_grid, with NumPy's zero sign fused in when the
        query allows it (min/max of a float variable, _fold_sign_ok) and the
        fold kernel the geometry takes can key it (the lean column fold with
        both reductions elementwise, or the LDS row fold).  Returns whether
        the sign was fused (else the zero-sign passes run)."""
        which = self._tie_which() if zs_ok else 0
        if which:
            try:
                engine.reduce_axes_grid(ctx, plan.batch, plan.mask_up.struct, g, fin_ptr, True, st,
                                        zero_sign=which)
                return True
            except NotImplementedError:
                pass   # another fold kernel: the sign comes from the tie passes
        engine.reduce_axes_grid(ctx, plan.batch, plan.mask_up.struct, g, fin_ptr, True, st)
        return False

    def _whole_chunk_grid(self, tables, final_shape, axes):
        """Every kept dim's output positions are whole chunks in coordinate
        order (position p -> coordinate p // chunk, local p % chunk), as
        pyas_reduce_axes_grid assumes."""
        blob = tables["blob"]
        for d, c in enumerate(self.ds.chunks):
            if d in axes:
                continue
            F = final_shape[d]
            if F != tables["n_coords"][d] * c:
                return False
            p = np.arange(F, dtype=np.int32)
            pc, pl = tables["pos_coord"][d], tables["pos_local"][d]
            if not (np.array_equal(blob[pc:pc + F], p // c) and np.array_equal(blob[pl:pl + F], p % c)):
                return False
        return True

    def _format_device(self, ctx, st, fin, n, shape, bufs=None):
        """``_format`` on the device (pyas_format_partials): only the
        result's values, mask (and counts in components mode) come back.
        ``bufs``: a dict that keeps the device result buffers for reuse."""
        dt = self.ds.dtype
        method = "sum" if (self._components and self._method == "mean") else self._method
        vdt = engine.format_dtype(dt, method)
        have = bufs.get((vdt.str, self._components)) if bufs is not None else None
        if have is None:
            have = (DeviceBuffer(ctx, max(n, 1) * vdt.itemsize), DeviceBuffer(ctx, max(n, 1)),
                    DeviceBuffer(ctx, max(n, 1) * 8) if self._components else None)
            if bufs is not None:
                bufs[(vdt.str, self._components)] = have
        vbuf, mbuf, cbuf = have
        engine.format_partials(ctx, dt, fin.ptr, n, method, vbuf.ptr, mbuf.ptr,
                               cbuf.ptr if cbuf is not None else None, st)
        vals = ctx.result_array(n, vdt)
        mask = ctx.result_array(n, np.bool_)
        ctx.d2h(vals, vbuf.ptr, st)
        ctx.d2h(mask, mbuf.ptr, st)
        if cbuf is not None:
            cnt = ctx.result_array(n, np.int64)
            ctx.d2h(cnt, cbuf.ptr, st)
        ctx.synchronize(st)
        out = np.ma.MaskedArray(vals.reshape(shape), mask=mask.reshape(shape))
        if self._components:
            nn = np.ma.MaskedArray(cnt.reshape(shape), mask=np.zeros(shape, dtype=bool))
            return {method: out, "n": nn}
        return out

    def _reduce_general(self, indexer, compressor, filters, axes):
        """Per-chunk selection objects and host-built segments: integer-
        dropped dims and vector fill/missing values."""
        ds = self.ds
        dt = ds.dtype
        chunk_list = list(indexer)
        final_shape = tuple(1 if i in axes else n for i, n in enumerate(indexer.shape))
        n_final = int(np.prod(final_shape))
        pdt = engine.partial_dtype(dt)
        if not chunk_list:
            final = np.zeros(n_final, dtype=pdt)
            return self._format(final.reshape(final_shape), final_shape)
        ctx, st, buf, offsets, fused = self._ingest([c for c, _ in chunk_list], compressor, filters)
        sels = [self._chunk_sel(projs) for _, projs in chunk_list]
        plan = ReductionPlan(ctx, dt, ds.chunks, buf.ptr, offsets, shuffle=fused, selections=sels,
                             missing=self.missing, round_to_var=True, stream=st)
        if len(axes) == ds.ndim:
            final = self._total(plan, st)
            return self._format(final.reshape(final_shape), final_shape)
        axes_mask = 0
        for a in axes:
            axes_mask |= 1 << a
        grid = self._grid_tables(chunk_list, axes, final_shape)
        if grid is not None:
            return self._grid_combine(ctx, st, plan, grid, axes, final_shape)
        # general case: per-chunk partial arrays, then a segmented device combine
        sizes, fidx = [], []
        for _, projs in chunk_list:
            pos = [p.out_pos if i not in axes else np.zeros(1, dtype=np.int64)
                   for i, p in enumerate(projs)]
            grids = np.meshgrid(*pos, indexing="ij")
            fidx.append(np.ravel_multi_index([g.reshape(-1) for g in grids], final_shape))
            sizes.append(grids[0].size)
        out_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        f_all = np.concatenate(fidx)
        order = np.argsort(f_all, kind="stable").astype(np.int64)
        seg = np.searchsorted(f_all[order], np.arange(n_final + 1)).astype(np.int64)
        axes_mask = 0
        for a in axes:
            axes_mask |= 1 << a
        meta = np.concatenate([out_off[:-1], order, seg])
        mbuf = DeviceBuffer(ctx, meta.nbytes)
        ctx.h2d(mbuf.ptr, meta, st)
        prec = engine.method_rec(self._method)   # compact per-output records (see _grid_partials)
        parts = DeviceBuffer(ctx, max(int(out_off[-1]), 1) * _lib.rec_nbytes(dt.itemsize, prec))
        fin = DeviceBuffer(ctx, max(n_final, 1) * _lib.PARTIAL_NBYTES)
        engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, axes_mask, mbuf.ptr, parts.ptr, st, rec=prec)
        engine.combine_segments(ctx, dt, parts.ptr, mbuf.ptr + 8 * len(chunk_list),
                                mbuf.ptr + 8 * (len(chunk_list) + order.size), n_final, fin.ptr,
                                True, st, rec=prec)
        which = self._tie_which()
        if which:   # NumPy's zero sign: per chunk output, then over each segment's layers
            which |= _lib.TIE_REC
            engine.tie_chunks(ctx, plan.batch, plan.mask_up.struct, plan.tie_geom(), axes_mask, which, mbuf.ptr,
                              parts.ptr, st)
            ncoord = [len({cc[d] for cc, _ in chunk_list}) for d in range(ds.ndim)]
            lr = zerosign.grid_lr([ncoord[d] if d in axes else final_shape[d] for d in range(ds.ndim)], set(axes))
            engine.tie_segments(ctx, dt, parts.ptr, mbuf.ptr + 8 * len(chunk_list),
                                mbuf.ptr + 8 * (len(chunk_list) + order.size), n_final, int(np.diff(seg).max()),
                                0, lr, which, fin.ptr, None, st)
        final = np.zeros(n_final, dtype=pdt)
        ctx.d2h(final, fin.ptr, st)
        ctx.synchronize(st)
        return self._format(final.reshape(final_shape), final_shape)

    def _grid_tables(self, chunk_list, axes, final_shape):
        """``_grid_from_dims`` for a materialised chunk list, when its chunks
        are the C-ordered product of per-dim projections; else None."""
        nd = self.ds.ndim
        seen = [dict() for _ in range(nd)]
        dims = [[] for _ in range(nd)]
        idx = np.empty((len(chunk_list), nd), dtype=np.int64)
        for k, (cc, projs) in enumerate(chunk_list):
            if len(projs) != nd:
                return None
            for d in range(nd):
                p = projs[d]
                if isinstance(p.chunk_sel, (int, np.integer)):
                    return None
                a = seen[d].get(cc[d])
                if a is None:
                    a = seen[d][cc[d]] = len(dims[d])
                    dims[d].append(p)
                idx[k, d] = a
        n_coords = [len(o) for o in dims]
        if int(np.prod(n_coords)) != len(chunk_list):
            return None
        if not (np.ravel_multi_index(idx.T, n_coords) == np.arange(len(chunk_list))).all():
            return None
        return self._grid_from_dims(dims, axes, final_shape)

    @staticmethod
    def _grid_from_dims(dims, axes, final_shape):
        """Tables of ``pyas_combine_grid`` from per-dim projections (chunks =
        their C-ordered product).  Returns ``(out_off, tables)``: ``out_off[n]``
        is chunk n's offset in the partial array (its kept-dims selection, C
        order); ``tables`` holds one int32 blob with, per kept dim, position
        -> coordinate index, position -> index inside that chunk's selection
        and coordinate -> selected count (offsets in int32 units)."""
        nd = len(dims)
        n_coords = [len(p) for p in dims]
        kept = [d for d in range(nd) if d not in axes]
        counts = {d: np.array([len(p.out_pos) for p in dims[d]], dtype=np.int64) for d in kept}
        n = int(np.prod(n_coords))
        idx = np.indices(n_coords).reshape(nd, n)
        sizes = np.ones(n, dtype=np.int64)
        for d in kept:
            sizes *= counts[d][idx[d]]
        out_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        parts, off = [], 0
        tables = {"n_coords": n_coords, "pos_coord": {}, "pos_local": {}, "coord_count": {},
                  "n_parts": int(sizes.sum())}
        for d in kept:
            F = final_shape[d]
            pc = np.full(F, -1, dtype=np.int32)
            pl = np.zeros(F, dtype=np.int32)
            for a, p in enumerate(dims[d]):
                o = np.asarray(p.out_pos, dtype=np.int64)
                pc[o] = a
                pl[o] = np.arange(o.size, dtype=np.int32)
            if (pc < 0).any():
                raise AssertionError("output positions not covered by the chunk projections")
            for name, arr in (("pos_coord", pc), ("pos_local", pl),
                              ("coord_count", counts[d].astype(np.int32))):
                tables[name][d] = off
                parts.append(arr)
                off += arr.size
        tables["blob"] = np.concatenate(parts) if parts else np.zeros(1, dtype=np.int32)
        return out_off, tables

    def _format(self, final, shape):
        """active.py:591-630 on combined partials."""
        dt = self.ds.dtype
        cnt = np.ascontiguousarray(final["count"]).astype(np.int64)
        if self._method in ("sum", "mean"):
            vals = final["sum"].astype(native(dt) if dt.kind == "f" else sum_dtype(dt))
        else:
            vals = final[self._method].astype(native(dt))
        out = np.ma.MaskedArray(np.ascontiguousarray(vals), mask=(cnt == 0))
        n = np.ma.MaskedArray(cnt, mask=np.zeros(shape, dtype=bool))
        if self._components:
            return {("sum" if self._method == "mean" else self._method): out, "n": n}
        if self._method == "mean":
            return out / n
        return out

    # -- method=None --------------------------------------------------------
    def _select(self, indexer, compressor, filters):
        if not any(m is not None and np.size(m) != 1 for m in self.missing):
            return self._select_scatter(indexer, compressor, filters)
        return self._select_general(indexer, compressor, filters)

    def _select_scatter(self, indexer, compressor, filters):
        """method=None over the whole query in one launch: every selected
        element is written by the device straight to its place in the
        C-ordered result (pyas_select_scatter), instead of per-chunk host
        placement at each chunk's out_selection."""
        ds = self.ds
        dt = ds.dtype
        dims = [list(d) for d in indexer.dim_indexers]
        nd = len(dims)
        n_coords = [len(p) for p in dims]
        n = int(np.prod(n_coords))
        out_shape = indexer.shape
        # output strides: C order over the kept dims, 0 for integer-dropped ones
        ostride = np.zeros(nd, dtype=np.int64)
        kept = [d for d in range(nd) if indexer.dim_indexers[d].kind != "int"]
        acc = 1
        for d in reversed(kept):
            ostride[d] = acc
            acc *= out_shape[kept.index(d)]
        ent, pos_parts, bases, pool_parts = [], [], [], []
        ppos = poolpos = 0
        for projs in dims:
            e = np.zeros((len(projs), 3), dtype=np.int32)
            b = np.zeros(len(projs), dtype=np.int32)
            for a, p in enumerate(projs):
                sl = p.chunk_sel
                if isinstance(sl, slice):
                    cnt = len(p.out_pos)
                    e[a] = (sl.start if cnt else 0, sl.step, cnt)
                    op = np.asarray(p.out_pos, dtype=np.int64)
                elif isinstance(sl, np.ndarray):
                    e[a] = (poolpos, 0, sl.size)
                    pool_parts.append(sl.astype(np.int32))
                    poolpos += sl.size
                    op = np.asarray(p.out_pos, dtype=np.int64)
                else:                                        # integer index: dropped dim
                    e[a] = (int(sl), 1, 1)
                    op = np.zeros(1, dtype=np.int64)
                b[a] = ppos
                pos_parts.append(op)
                ppos += op.size
            ent.append(e)
            bases.append(b)
        nd_native = native(dt)
        if n == 0 or int(np.prod(out_shape)) == 0:
            return np.ma.MaskedArray(np.zeros(out_shape, dtype=dt))
        idx = np.indices(n_coords).reshape(nd, n)
        table = np.zeros((n, _lib.MAX_DIMS, 3), dtype=np.int32)
        table[:, :, 1] = 1
        table[:, :, 2] = 1
        cbase = np.zeros((n, nd), dtype=np.int32)
        coords = np.zeros((n, nd), dtype=np.int64)
        for d in range(nd):
            table[:, d, :] = ent[d][idx[d]]
            cbase[:, d] = bases[d][idx[d]]
            coords[:, d] = np.array([p.chunk_ix for p in dims[d]], dtype=np.int64)[idx[d]]
        pool = np.concatenate(pool_parts) if pool_parts else np.zeros(1, dtype=np.int32)
        pos = np.concatenate(pos_parts)
        ctx, st, buf, offsets, fused = self._ingest(coords, compressor, filters)
        full = _all_full(table, ds.chunks)
        plan = ReductionPlan(ctx, dt, ds.chunks, buf.ptr, offsets, shuffle=fused,
                             sel_table=None if full else table, index_pool=None if full else pool,
                             missing=self.missing, stream=st)
        total = int(np.prod(out_shape))
        pb = DeviceBuffer(ctx, pos.nbytes)
        ctx.h2d(pb.ptr, pos, st)
        cb = DeviceBuffer(ctx, cbase.nbytes)
        ctx.h2d(cb.ptr, np.ascontiguousarray(cbase), st)
        sc = _lib.Scatter()
        sc.pos, sc.chunk_base = pb.ptr, cb.ptr
        for d in range(nd):
            sc.out_stride[d] = int(ostride[d])
        vals = ctx.result_array(total, nd_native)
        msk = ctx.result_array(total, np.uint8)
        vb = DeviceBuffer(ctx, vals.nbytes)
        mb = DeviceBuffer(ctx, msk.nbytes)
        engine.select_scatter(ctx, plan.batch, plan.mask_up.struct, sc, vb.ptr, mb.ptr, st)
        ctx.d2h(vals, vb.ptr, st)
        ctx.d2h(msk, mb.ptr, st)
        ctx.synchronize(st)
        out_vals = vals.reshape(out_shape).astype(dt, copy=False)
        out_mask = msk.reshape(out_shape).view(bool)
        if out_mask.any():
            return np.ma.MaskedArray(out_vals, mask=out_mask)
        return np.ma.MaskedArray(out_vals)

    def _select_general(self, indexer, compressor, filters):
        """method=None with vector fill/missing values (per-chunk selections)."""
        ds = self.ds
        dt = ds.dtype
        chunk_list = list(indexer)
        out_vals = np.zeros(indexer.shape, dtype=dt)
        out_mask = np.zeros(indexer.shape, dtype=bool)
        if chunk_list:
            ctx, st, buf, offsets, fused = self._ingest([c for c, _ in chunk_list], compressor, filters)
            sels = [self._chunk_sel(projs) for _, projs in chunk_list]
            plan = ReductionPlan(ctx, dt, ds.chunks, buf.ptr, offsets, shuffle=fused,
                                 selections=sels, missing=self.missing, stream=st)
            sizes = np.array([s.n_selected for s in sels], dtype=np.int64)
            off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
            total = int(off[-1])
            nd = native(dt)
            vals = np.zeros(max(total, 1), dtype=nd)
            msk = np.zeros(max(total, 1), dtype=np.uint8)
            ob = DeviceBuffer(ctx, off.nbytes)
            ctx.h2d(ob.ptr, off, st)
            vb = DeviceBuffer(ctx, vals.nbytes)
            mb = DeviceBuffer(ctx, msk.nbytes)
            engine.select_chunks(ctx, plan.batch, plan.mask_up.struct, ob.ptr, vb.ptr, mb.ptr, st)
            ctx.d2h(vals, vb.ptr, st)
            ctx.d2h(msk, mb.ptr, st)
            ctx.synchronize(st)
            for c, (_, projs) in enumerate(chunk_list):
                block = slice(int(off[c]), int(off[c + 1]))
                where = np.ix_(*[p.out_pos for p in projs if not isinstance(p.chunk_sel, (int, np.integer))])
                out_vals[where] = vals[block].reshape(sels[c].shape)
                out_mask[where] = msk[block].reshape(sels[c].shape).astype(bool)
        if out_mask.any():
            return np.ma.MaskedArray(out_vals, mask=out_mask)
        return np.ma.MaskedArray(out_vals)
