"""GPU zlib inflate (row f3): ``pyas_inflate`` over a batch of chunk streams.

The reference decompresses each chunk on the host with
``numcodecs.Zlib.decode`` -> ``zlib.decompress`` (built at
``activestorage/hdf2numcodec.py:34-35``, applied at
``activestorage/storage.py:119-120``).  Here the compressed chunk bytes of a
whole query are uploaded once and inflated device to device, one wave per
stream, straight into the chunk-major buffer the reduce kernels read.

Failures are raised as ``zlib.error`` with zlib's own wording, the exception
``zlib.decompress`` raises for the same stream.
"""
from __future__ import annotations

import zlib

import numpy as np

from . import _lib
from .device import Context, DeviceBuffer

# pyas_inflate_status -> (zlib return code, zlib message)
_MESSAGES = {
    1: (-3, "incorrect header check"),
    2: (2, "need dictionary"),
    3: (-3, "invalid block type"),
    4: (-3, "invalid stored block lengths"),
    5: (-3, "invalid code lengths set"),
    6: (-3, "invalid literal/length or distance code"),
    7: (-3, "invalid distance too far back"),
    8: (-5, "incomplete or truncated stream"),
    9: (-3, "incorrect data check"),
}


def raise_for_status(status: np.ndarray, out_sizes: np.ndarray, capacity: np.ndarray,
                     base: int = 0) -> None:
    """Raise the ``zlib.error`` zlib.decompress would give for the first failed
    stream; an output larger than the caller's capacity is a ValueError (the
    reference fails reshaping the oversized chunk, storage.py:57-62)."""
    bad = np.nonzero(status)[0]
    if bad.size == 0:
        return
    c = int(bad[0])
    code = int(status[c])
    if code == 10:
        raise ValueError(f"chunk {base + c} inflates to more than its {int(capacity[c])} bytes")
    rc, msg = _MESSAGES.get(code, (-3, f"inflate status {code}"))
    if rc == 2:
        raise zlib.error(f"Error {rc} while decompressing data")
    raise zlib.error(f"Error {rc} while decompressing data: {msg}")


class InflateBatch:
    """Device-side descriptors for one launch of ``pyas_inflate``.

    src_offsets/src_sizes locate the compressed streams in ``src_ptr``;
    dst_offsets/capacity give each stream's output slot in ``dst_ptr``.
    """

    def __init__(self, ctx: Context, src_offsets, src_sizes, dst_offsets, capacity, scratch: bool = False):
        self.ctx = ctx
        self.n = int(len(src_offsets))
        self.capacity = np.ascontiguousarray(capacity, dtype=np.int64)
        meta = np.concatenate([np.asarray(src_offsets, np.int64), np.asarray(src_sizes, np.int64),
                               np.asarray(dst_offsets, np.int64), self.capacity])
        # [src_off | src_size | dst_off | cap | out_sizes (int64) | status (int32)]
        nbytes = meta.nbytes + self.n * 8 + self.n * 4
        # scratch: reuse the calling thread's growable buffer (per-chunk drop-in)
        self.buf = ctx.thread_buffer("inflate_meta", nbytes) if scratch else DeviceBuffer(ctx, nbytes)
        self._meta = meta
        self.out_sizes = np.zeros(self.n, dtype=np.int64)
        self.status = np.zeros(self.n, dtype=np.int32)

    def launch(self, src_ptr: int, dst_ptr: int, stream) -> None:
        n, p = self.n, self.buf.ptr
        if n == 0:
            return
        self.ctx.h2d(p, self._meta, stream)
        _lib.check(self.ctx.lib.pyas_inflate(self.ctx.handle, src_ptr, p, p + 8 * n, n, dst_ptr,
                                             p + 16 * n, p + 24 * n, p + 32 * n, p + 40 * n, stream),
                   "pyas_inflate")

    def results(self, stream):
        """Synchronise and return (out_sizes, status)."""
        if self.n:
            p = self.buf.ptr
            self.ctx.d2h(self.out_sizes, p + 32 * self.n, stream)
            self.ctx.d2h(self.status, p + 40 * self.n, stream)
        self.ctx.synchronize(stream)
        return self.out_sizes, self.status

    def check(self, stream, exact: bool = True, base: int = 0) -> np.ndarray:
        """Synchronise, raise like zlib on failure, and (``exact``) require every
        stream to fill its slot exactly (a chunk's decoded size is fixed)."""
        sizes, status = self.results(stream)
        raise_for_status(status, sizes, self.capacity, base)
        if exact and self.n and (sizes != self.capacity).any():
            c = int(np.nonzero(sizes != self.capacity)[0][0])
            raise ValueError(f"chunk {base + c} inflated to {int(sizes[c])} bytes, "
                             f"expected {int(self.capacity[c])}")
        return sizes


def is_zlib(compression) -> bool:
    return getattr(compression, "codec_id", None) == "zlib"


def inflate_chunk(ctx: Context, raw, dst_ptr: int, nbytes: int, stream) -> None:
    """Inflate one chunk's zlib stream into ``dst_ptr`` (``nbytes`` exactly),
    through the calling thread's scratch buffers; raises like zlib."""
    src = np.frombuffer(memoryview(raw), dtype=np.uint8)
    sbuf = ctx.thread_buffer("inflate_src", max(src.size, 16))
    ctx.h2d(sbuf.ptr, src, stream)
    b = InflateBatch(ctx, [0], [src.size], [0], [nbytes], scratch=True)
    b.launch(sbuf.ptr, dst_ptr, stream)
    b.check(stream)


def pack_streams(streams, align: int = 16):
    """Concatenate byte strings into one uint8 array; returns (host, offsets, sizes)."""
    sizes = np.array([len(s) for s in streams], dtype=np.int64)
    padded = -(-sizes // align) * align
    offsets = np.concatenate([[0], np.cumsum(padded)[:-1]]).astype(np.int64) if len(streams) else sizes
    host = np.zeros(max(int(padded.sum()), 1), dtype=np.uint8)
    for o, s in zip(offsets, streams):
        host[o:o + len(s)] = np.frombuffer(memoryview(s), dtype=np.uint8)
    return host, offsets, sizes


def inflate_many(ctx: Context, streams, capacity, stream=None, src_align: int = 16,
                 dst_align: int = 256) -> list:
    """Host convenience (tests, drop-in): inflate byte strings on the device and
    return the decoded bytes of each.  ``capacity`` is an int or per-stream list;
    the alignments place streams and output slots in their device buffers."""
    n = len(streams)
    if n == 0:
        return []
    cap = np.broadcast_to(np.asarray(capacity, dtype=np.int64), (n,)).copy()
    host, offs, sizes = pack_streams(streams, src_align)
    slot = -(-cap // dst_align) * dst_align
    dst_off = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.int64)
    st = ctx.thread_stream() if stream is None else stream
    src = DeviceBuffer(ctx, host.nbytes)
    dst = DeviceBuffer(ctx, max(int(slot.sum()), 1))
    ctx.h2d(src.ptr, host, st)
    b = InflateBatch(ctx, offs, sizes, dst_off, cap)
    b.launch(src.ptr, dst.ptr, st)
    out_sizes, status = b.results(st)
    raise_for_status(status, out_sizes, cap)
    out = np.zeros(max(int(slot.sum()), 1), dtype=np.uint8)
    ctx.d2h(out, dst.ptr, st)
    ctx.synchronize(st)
    return [out[o:o + s].tobytes() for o, s in zip(dst_off, out_sizes)]
