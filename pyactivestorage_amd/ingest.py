"""Host ingest (row f2): file byte ranges straight into device memory.

The reference opens the file and reads every chunk separately
(``activestorage/storage.py:51-53`` ``open`` + ``read_block`` at
``:156-162``), once per chunk on a 30-thread pool (``active.py:557-572``).
:func:`read_ranges` hands a whole query's ranges to ``pyas_read_ranges``
(``include/pyas.h``): native reader threads ``pread`` into pinned staging
slots, and each filled slot is copied H2D on the caller's stream while the
next ones are read.  Opening the file stays in Python, so a missing file
raises ``FileNotFoundError`` exactly where the reference's ``open`` does.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib
from .device import Context

DEFAULT_THREADS = 16


def read_ranges(ctx: Context, path: str, file_offsets, sizes, dst_ptr: int, dst_offsets,
                stream=None, threads: int = DEFAULT_THREADS) -> int:
    """Read ``file[file_offsets[i] : + sizes[i]]`` into ``dst_ptr + dst_offsets[i]``
    (device) for every i.  Returns the bytes read.  The copies are enqueued
    on ``stream``; work queued after them on that stream sees the data."""
    foff = np.ascontiguousarray(file_offsets, dtype=np.int64)
    size = np.ascontiguousarray(sizes, dtype=np.int64)
    doff = np.ascontiguousarray(dst_offsets, dtype=np.int64)
    if not (foff.shape == size.shape == doff.shape) or foff.ndim != 1:
        raise ValueError("file_offsets, sizes and dst_offsets must be 1-D and of equal length")
    fd = os.open(path, os.O_RDONLY)
    try:
        _lib.check(ctx.lib.pyas_read_ranges(ctx.handle, fd, int(foff.size), foff.ctypes.data,
                                            size.ctypes.data, dst_ptr, doff.ctypes.data,
                                            int(threads), stream),
                   f"pyas_read_ranges({path})")
    finally:
        os.close(fd)
    return int(size.sum())


def set_slots(ctx: Context, n_slots: int, slot_bytes: int) -> None:
    """Resize the pinned staging ring (default 16 x 64 MiB)."""
    _lib.check(ctx.lib.pyas_ctx_set_ingest_slots(ctx.handle, int(n_slots), int(slot_bytes)),
               "pyas_ctx_set_ingest_slots")


def read_ranges_zlib(ctx: Context, path: str, file_offsets, sizes, dst_ptr: int, dst_offsets,
                     out_bytes: int, stream=None, threads: int = DEFAULT_THREADS, reshape=None) -> int:
    """Host inflate straight into the pinned ring (``pyas_read_ranges_zlib``):
    range i of the file is one zlib stream that must inflate to exactly
    ``out_bytes`` bytes at ``dst_ptr + dst_offsets[i]`` (device), the same
    bytes ``zlib.decompress`` gives (storage.py:119-120).  A stream that fails
    is decompressed again with ``zlib.decompress`` so the caller gets zlib's
    own ``zlib.error``; a wrong output size raises ValueError as the
    reference's reshape does (storage.py:57-62; ``reshape`` = (itemsize,
    chunk shape) words it the same way).  Returns the bytes read."""
    import zlib

    foff = np.ascontiguousarray(file_offsets, dtype=np.int64)
    size = np.ascontiguousarray(sizes, dtype=np.int64)
    doff = np.ascontiguousarray(dst_offsets, dtype=np.int64)
    if not (foff.shape == size.shape == doff.shape) or foff.ndim != 1:
        raise ValueError("file_offsets, sizes and dst_offsets must be 1-D and of equal length")
    status = np.zeros(foff.size, dtype=np.int32)
    fd = os.open(path, os.O_RDONLY)
    try:
        _lib.check(ctx.lib.pyas_read_ranges_zlib(ctx.handle, fd, int(foff.size), foff.ctypes.data,
                                                 size.ctypes.data, dst_ptr, doff.ctypes.data, int(out_bytes),
                                                 status.ctypes.data, int(threads), stream),
                   f"pyas_read_ranges_zlib({path})")
        bad = np.nonzero(status)[0]
        if bad.size:
            i = int(bad[0])
            raw = os.pread(fd, int(size[i]), int(foff[i]))
            out = zlib.decompress(raw)       # raises zlib's error for a broken stream
            if reshape is not None:          # (itemsize, chunk shape): the reference's reshape error
                raise ValueError(f"cannot reshape array of size {len(out) // reshape[0]} into shape {reshape[1]}")
            raise ValueError(f"chunk stream {i} inflates to {len(out)} bytes, not the chunk's {int(out_bytes)}")
    finally:
        os.close(fd)
    return int(size.sum())
