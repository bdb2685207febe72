"""Device context, streams and device buffers over the C ABI.

One ``Context`` per GPU (process-wide, created lazily).  Every calling thread
gets its own HIP stream so that concurrent ``reduce_chunk`` calls from the
reference's 30-thread pool (``activestorage/active.py:557-572``) never share
scratch memory; the C library keys its scratch by stream.
"""
from __future__ import annotations

import ctypes
import threading

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


class Context:
    """A ``pyas_ctx`` bound to one device."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        self.device = int(device)
        h = ctypes.c_void_p()
        _lib.check(self.lib.pyas_ctx_create(self.device, ctypes.byref(h)), "pyas_ctx_create")
        self.handle = h.value
        self._tls = threading.local()

    # -- streams -------------------------------------------------------------
    def thread_stream(self) -> int:
        s = getattr(self._tls, "stream", None)
        if s is None:
            p = ctypes.c_void_p()
            _lib.check(self.lib.pyas_stream_create(self.handle, ctypes.byref(p)),
                       "pyas_stream_create")
            s = self._tls.stream = p.value
        return s

    def thread_aux_stream(self, k: int = 0) -> int:
        """Extra stream ``k`` of the calling thread (ingest copies and inflate
        groups that overlap device work queued on :meth:`thread_stream`)."""
        aux = getattr(self._tls, "aux_streams", None)
        if aux is None:
            aux = self._tls.aux_streams = {}
        s = aux.get(k)
        if s is None:
            p = ctypes.c_void_p()
            _lib.check(self.lib.pyas_stream_create(self.handle, ctypes.byref(p)),
                       "pyas_stream_create")
            s = aux[k] = p.value
        return s

    def stream_wait(self, waiter: int, waitee: int) -> None:
        """Later work on ``waiter`` waits for everything queued on ``waitee``."""
        _lib.check(self.lib.pyas_stream_wait(self.handle, waiter, waitee), "pyas_stream_wait")

    def synchronize(self, stream: int | None) -> None:
        _lib.check(self.lib.pyas_stream_synchronize(self.handle, stream), "pyas_stream_synchronize")
        self._tls.pending = []

    # -- per-thread growable scratch buffers ---------------------------------
    def thread_buffer(self, slot: str, nbytes: int) -> DeviceBuffer:
        bufs = getattr(self._tls, "bufs", None)
        if bufs is None:
            bufs = self._tls.bufs = {}
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
        hb = getattr(self._tls, "host_buf", None)
        if hb is None or hb[1] < nbytes:
            if hb is not None:
                self.synchronize(self.thread_stream())
                _lib.check(self.lib.pyas_host_free(self.handle, hb[0]), "pyas_host_free")
            size = max(int(nbytes), 1 << 20)
            p = ctypes.c_void_p()
            _lib.check(self.lib.pyas_host_alloc(self.handle, size, ctypes.byref(p)), "pyas_host_alloc")
            arr = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p.value))
            hb = self._tls.host_buf = (p.value, size, arr)
        return hb[2]

    # -- copies --------------------------------------------------------------
    def h2d(self, dst_ptr: int, host: np.ndarray, stream: int | None) -> None:
        """Async copy; the host array is kept alive until the next
        ``synchronize`` of this thread (HIP may read pageable memory late)."""
        host = np.ascontiguousarray(host)
        _lib.check(self.lib.pyas_memcpy_h2d(self.handle, dst_ptr, host.ctypes.data, host.nbytes, stream),
                   "pyas_memcpy_h2d")
        pending = getattr(self._tls, "pending", None)
        if pending is None:
            pending = self._tls.pending = []
        pending.append(host)

    def d2h(self, host: np.ndarray, src_ptr: int, stream: int | None) -> None:
        assert host.flags.c_contiguous
        _lib.check(self.lib.pyas_memcpy_d2h(self.handle, host.ctypes.data, src_ptr, host.nbytes, stream),
                   "pyas_memcpy_d2h")

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
