"""Device context, streams and device buffers over the C ABI.

One ``Context`` per GPU (process-wide, created lazily).  A calling thread
that needs its own HIP stream (``Active`` queries, the per-call fallback of
the drop-in) gets one, plus scratch keyed by that stream in the C library;
both are released when the thread ends.  The drop-in's common path
(``storage.reduce_chunk`` from the reference's 30-thread pool,
``activestorage/active.py:557-572``) instead goes through the context's one
coalescer (``pyas_coalesced_reduce``) and holds no per-thread device state.
"""
from __future__ import annotations

import ctypes
import os
import threading
import warnings
import weakref

import numpy as np

from . import _lib

_ctx_lock = threading.Lock()
_contexts: dict[int, "Context"] = {}


def device_count() -> int:
    n = ctypes.c_int(0)
    _lib.check(_lib.load().pyas_device_count(ctypes.byref(n)), "pyas_device_count")
    return n.value


class DeviceBuffer:
    """Owning device allocation made through ``pyas_malloc``."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _lib.check(ctx.lib.pyas_malloc(ctx.handle, max(self.nbytes, 1), ctypes.byref(p)),
                   "pyas_malloc")
        self.ptr = p.value

    def free(self):
        if self.ptr:
            self.ctx.lib.pyas_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.free()
        except Exception:
            pass


class _ThreadResources:
    """What one thread holds on one context: its HIP streams, growable device
    scratch buffers, pinned staging buffer and the pageable arrays its async
    copies still read.  Released when the thread ends (its ``threading.local``
    entry is dropped): the streams are synchronised, the buffers freed and
    the streams destroyed, which also frees the C library's per-stream scratch.
    The reference builds a new 30-thread pool per query (active.py:557), so
    per-thread resources must not outlive their thread."""

    def __init__(self, ctx: "Context"):
        # the finalizer holds `state`, never `self`
        self.state = state = {"stream": None, "aux": {}, "bufs": {}, "host": None, "pending": {}}
        fin = weakref.finalize(self, _release_thread, ctx, state)
        fin.atexit = False   # at interpreter exit the process releases everything


def _release_thread(ctx: "Context", state) -> None:
    lib, h = ctx.lib, ctx.handle
    streams = ([state["stream"]] if state["stream"] else []) + list(state["aux"].values())
    for s in streams:
        lib.pyas_stream_synchronize(h, s)
    for b in state["bufs"].values():
        b.free()
    if state["host"] is not None:
        lib.pyas_host_free(h, state["host"][0])
        ctx._count(pinned=-state["host"][1])
    for s in streams:
        lib.pyas_stream_destroy(h, s)
        ctx._count(streams=-1)
    state.clear()


class _ResultPool:
    """Pinned host blocks for query results that come back from the device
    (``Active``'s formatted values and mask): a D2H copy into pinned memory
    is DMA at the PCIe rate, into a fresh pageable ``np.empty`` it is staged
    by the runtime.  A block is leased to the array built on it and returns
    to the pool's free list when that array (and every view of it) is
    collected.  Blocks are power-of-two sized; at most ``cap`` bytes are
    pinned, beyond that callers get pageable arrays."""

    MIN_BYTES = 64 << 10   # smaller results: pageable (the copy is latency-bound)

    def __init__(self, ctx: "Context", cap: int):
        self.ctx, self.cap = ctx, int(cap)
        self.lock = threading.Lock()
        self.free: dict[int, list[int]] = {}
        self.pinned = 0          # bytes pinned by the pool (leased + free)

    def array(self, n: int, dtype) -> np.ndarray:
        dt = np.dtype(dtype)
        nbytes = int(n) * dt.itemsize
        if nbytes < self.MIN_BYTES or self.cap <= 0:
            return np.empty(n, dtype=dt)
        size = 1 << (nbytes - 1).bit_length()
        with self.lock:
            blocks = self.free.get(size)
            ptr = blocks.pop() if blocks else None
            if ptr is None:
                if self.pinned + size > self.cap:
                    return np.empty(n, dtype=dt)
                p = ctypes.c_void_p()
                _lib.check(self.ctx.lib.pyas_host_alloc(self.ctx.handle, size, ctypes.byref(p)),
                           "pyas_host_alloc")
                ptr = p.value
                self.pinned += size
        raw = (ctypes.c_uint8 * nbytes).from_address(ptr)
        raw._lease = _Lease(self, ptr, size)
        return np.frombuffer(raw, dtype=dt, count=n)

    def put(self, ptr: int, size: int) -> None:
        with self.lock:
            self.free.setdefault(size, []).append(ptr)


class _Lease:
    """Returns a pinned block to its pool when the result array is gone."""

    __slots__ = ("pool", "ptr", "size")

    def __init__(self, pool: _ResultPool, ptr: int, size: int):
        self.pool, self.ptr, self.size = pool, ptr, size

    def __del__(self):
        try:
            self.pool.put(self.ptr, self.size)
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


_TIE_WARNED: set = set()
_TIE_WARN_LOCK = threading.Lock()


def host_tie_rules():
    """[(ABI dtype code, "f4"/"f8", TieRule or None)] for this host.  When
    no rule reproduces NumPy's choice of +0.0/-0.0 for a dtype (zerosign.py
    derives it from NumPy at start-up), a zero min/max of that dtype keeps
    the sign the device's reduction gives, which may differ from
    storage.py's; that is reported once per process and dtype as a
    RuntimeWarning and in ``Context.tie_signs_exact``."""
    from . import zerosign
    out = []
    for code, dt in ((_lib.F32, "f4"), (_lib.F64, "f8")):
        rule = zerosign.tie_rule(dt)
        if rule is None:
            with _TIE_WARN_LOCK:
                first = dt not in _TIE_WARNED
                _TIE_WARNED.add(dt)
            if first:
                warnings.warn(f"pyactivestorage_amd: no zero-sign rule reproduces this host's NumPy for {dt}; "
                              f"the sign of a zero min/max of {dt} data may differ from storage.py's "
                              f"(Context.tie_signs_exact)", RuntimeWarning, stacklevel=3)
        out.append((code, dt, rule))
    return out


class Context:
    """A ``pyas_ctx`` bound to one device."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        self.device = int(device)
        h = ctypes.c_void_p()
        _lib.check(self.lib.pyas_ctx_create(self.device, ctypes.byref(h)), "pyas_ctx_create")
        self.handle = h.value
        self._set_tie_rules()
        slots = os.environ.get("PYAS_INGEST_SLOTS")   # e.g. "64x16": 64 pinned slots of 16 MiB
        if slots:
            n, mib = (int(x) for x in slots.lower().split("x"))
            _lib.check(self.lib.pyas_ctx_set_ingest_slots(self.handle, n, mib << 20), "pyas_ctx_set_ingest_slots")
        self._tls = threading.local()
        self._stats_lock = threading.Lock()
        self.live_streams = 0        # per-thread streams currently alive
        self.pinned_bytes = 0        # per-thread pinned staging currently alive
        self._coalescer = None
        # PYAS_RESULT_PINNED_MIB: pinned bytes for result arrays (0: pageable)
        self._results = _ResultPool(self, int(os.environ.get("PYAS_RESULT_PINNED_MIB", "256")) << 20)

    def _set_tie_rules(self):
        """NumPy's zero-sign tie rule of this host for f32/f64 (zerosign.py),
        so the device returns the same +0.0/-0.0 as storage.py:99-100.
        ``tie_signs_exact[dtype]`` says whether that holds on this host."""
        self.tie_signs_exact = {}
        for code, dt, rule in host_tie_rules():
            self.tie_signs_exact[dt] = rule is not None
            if rule is None:
                continue
            r = _lib.TieRule()
            r.lanes, r.piece, r.acc = rule.lanes, rule.piece, rule.acc
            for lane, rank in enumerate(rule.rank):
                r.rank[lane] = rank
            for k, rank in enumerate(rule.acc_rank):
                r.acc_rank[k] = rank
            _lib.check(self.lib.pyas_ctx_set_tie_rule(self.handle, code, ctypes.byref(r)), "set_tie_rule")

    def _count(self, streams=0, pinned=0):
        with self._stats_lock:
            self.live_streams += streams
            self.pinned_bytes += pinned

    def _res(self):
        r = getattr(self._tls, "res", None)
        if r is None:
            r = self._tls.res = _ThreadResources(self)
        return r.state

    def _new_stream(self) -> int:
        p = ctypes.c_void_p()
        _lib.check(self.lib.pyas_stream_create(self.handle, ctypes.byref(p)), "pyas_stream_create")
        self._count(streams=1)
        return p.value

    # -- streams -------------------------------------------------------------
    def thread_stream(self) -> int:
        st = self._res()
        if st["stream"] is None:
            st["stream"] = self._new_stream()
        return st["stream"]

    def thread_aux_stream(self, k: int = 0) -> int:
        """Extra stream ``k`` of the calling thread (ingest copies and inflate
        groups that overlap device work queued on :meth:`thread_stream`)."""
        aux = self._res()["aux"]
        s = aux.get(k)
        if s is None:
            s = aux[k] = self._new_stream()
        return s

    def stream_wait(self, waiter: int, waitee: int) -> None:
        """Later work on ``waiter`` waits for everything queued on ``waitee``."""
        _lib.check(self.lib.pyas_stream_wait(self.handle, waiter, waitee), "pyas_stream_wait")

    def synchronize(self, stream: int | None) -> None:
        _lib.check(self.lib.pyas_stream_synchronize(self.handle, stream), "pyas_stream_synchronize")
        pend = getattr(self._tls, "res", None)
        if pend is not None:
            pend.state["pending"].pop(stream, None)

    # -- per-thread growable scratch buffers ---------------------------------
    def thread_buffer(self, slot: str, nbytes: int) -> DeviceBuffer:
        bufs = self._res()["bufs"]
        b = bufs.get(slot)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                self.synchronize(self.thread_stream())
                b.free()
            b = bufs[slot] = DeviceBuffer(self, max(int(nbytes), 256))
        return b

    def thread_host_buffer(self, nbytes: int) -> np.ndarray:
        """Per-thread pinned host staging (uint8, at least ``nbytes``); H2D
        copies from it are DMA.  Reused by the thread's next call: callers
        synchronize the thread stream before refilling it."""
        st = self._res()
        hb = st["host"]
        if hb is None or hb[1] < nbytes:
            if hb is not None:
                self.synchronize(self.thread_stream())
                _lib.check(self.lib.pyas_host_free(self.handle, hb[0]), "pyas_host_free")
                self._count(pinned=-hb[1])
                st["host"] = None
            size = max(int(nbytes), 1 << 20)
            p = ctypes.c_void_p()
            _lib.check(self.lib.pyas_host_alloc(self.handle, size, ctypes.byref(p)), "pyas_host_alloc")
            self._count(pinned=size)
            arr = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p.value))
            hb = st["host"] = (p.value, size, arr)
        return hb[2]

    def result_array(self, n: int, dtype) -> np.ndarray:
        """A host array of ``n`` elements for a device result to be copied
        into: pinned (leased from the context's pool) when large enough."""
        return self._results.array(n, dtype)

    # -- copies --------------------------------------------------------------
    def h2d(self, dst_ptr: int, host: np.ndarray, stream: int | None) -> None:
        """Async copy; the host array is kept alive until ``stream`` is next
        synchronised through this context (HIP may read pageable memory late)."""
        host = np.ascontiguousarray(host)
        _lib.check(self.lib.pyas_memcpy_h2d(self.handle, dst_ptr, host.ctypes.data, host.nbytes, stream),
                   "pyas_memcpy_h2d")
        self._res()["pending"].setdefault(stream, []).append(host)

    def d2h(self, host: np.ndarray, src_ptr: int, stream: int | None) -> None:
        assert host.flags.c_contiguous
        _lib.check(self.lib.pyas_memcpy_d2h(self.handle, host.ctypes.data, src_ptr, host.nbytes, stream),
                   "pyas_memcpy_d2h")

    # -- the per-chunk drop-in's batching runtime ------------------------------
    def coalescer(self) -> int:
        """Handle of this device's ``pyas_coalescer`` (created on first use,
        lives as long as the process: one dispatcher thread, one pinned ring)."""
        c = self._coalescer
        if c is None:
            with self._stats_lock:
                if self._coalescer is None:
                    p = ctypes.c_void_p()
                    _lib.check(self.lib.pyas_coalescer_create(self.handle, 0, 0, ctypes.byref(p)),
                               "pyas_coalescer_create")
                    self._coalescer = p.value
                c = self._coalescer
        return c

    def coalescer_stats(self) -> dict:
        s = (ctypes.c_int64 * 8)()
        if self._coalescer is not None:
            _lib.check(self.lib.pyas_coalescer_stats(self._coalescer, s), "pyas_coalescer_stats")
        return {"batches": s[0], "chunks": s[1], "largest": s[2], "busy_s": s[3] * 1e-9,
                "read_s": s[4] * 1e-9, "wait_s": s[5] * 1e-9, "gpu_s": s[6] * 1e-9,
                "handed_back": s[7]}

    def set_tile_bytes(self, nbytes: int) -> None:
        _lib.check(self.lib.pyas_ctx_set_tile_bytes(self.handle, int(nbytes)), "set_tile_bytes")

    def set_fold_min_blocks(self, n: int) -> None:
        """Workgroup floor of the in-kernel layer fold (0 = default 2048)."""
        _lib.check(self.lib.pyas_ctx_set_fold_min_blocks(self.handle, int(n)), "set_fold_min_blocks")

    def set_chained_combine(self, on: bool) -> None:
        """Fold tiles -> chunks -> total in the reduce kernel's tail (default)
        or in separate combine launches; results are bit-identical."""
        _lib.check(self.lib.pyas_ctx_set_chained_combine(self.handle, 1 if on else 0),
                   "set_chained_combine")


def get_context(device: int = 0) -> Context:
    with _ctx_lock:
        c = _contexts.get(device)
        if c is None:
            c = _contexts[device] = Context(device)
        return c
