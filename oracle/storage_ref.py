"""NumPy restatement of PyActiveStorage's local chunk-reduction path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the GPU product never
imports this module.  Every function cites the reference code it restates;
paths are relative to the reference repository (NCAS-CMS/PyActiveStorage,
snapshot 2026-07-23, ``activestorage/__init__.py:5`` version 0.4.0).

Third-party arithmetic restated here (absent from the build image):

* ``numcodecs.Shuffle.decode`` (numcodecs 0.16.5, pinned in the reference's
  ``conda-linux-64.lock``; call site ``activestorage/hdf2numcodec.py:36-37`` ->
  ``activestorage/storage.py:121-122``).  Published algorithm: the encoded
  buffer holds byte-plane ``b`` of every element contiguously, so decoded byte
  ``i*es + b`` = encoded byte ``b*n + i`` with ``n = len // es``.  Pinned
  byte-exact against libhdf5's own H5Z shuffle decode (see
  ``tests/golden/extract_h5.py``).
* ``numcodecs.Zlib.decode`` == ``zlib.decompress`` of the same stream.
"""
from __future__ import annotations

import zlib

import numpy as np

__all__ = [
    "Zlib", "Shuffle", "unshuffle", "read_block", "filter_pipeline",
    "decode_chunk", "mask_missing", "reduce_chunk", "reduce_chunk_bytes",
    "combine_partials",
]


# ----------------------------------------------------------------------------
# Codecs (numcodecs restatements; decode side only)
# ----------------------------------------------------------------------------
class Zlib:
    """Restates ``numcodecs.Zlib`` as built at ``hdf2numcodec.py:34-35``."""

    codec_id = "zlib"

    def __init__(self, level=1):
        self.level = level

    def decode(self, buf):
        return zlib.decompress(bytes(buf))


def unshuffle(buf, elementsize):
    """HDF5/numcodecs byte un-shuffle (numcodecs 0.16.5 ``Shuffle.decode``).

    ``out[i*es + b] = in[b*n + i]`` for ``n = len(buf) // es``.  numcodecs
    leaves the trailing ``len % es`` bytes of its zero-initialised output
    untouched (HDF5 copies them); only ``len % es == 0`` occurs on the path.
    """
    raw = np.frombuffer(memoryview(buf), dtype=np.uint8)
    es = int(elementsize)
    if es <= 1:
        return raw.copy()
    n = raw.size // es
    out = np.zeros(raw.size, dtype=np.uint8)
    out[: n * es] = raw[: n * es].reshape(es, n).T.reshape(-1)
    return out


class Shuffle:
    """Restates ``numcodecs.Shuffle`` as built at ``hdf2numcodec.py:36-37``."""

    codec_id = "shuffle"

    def __init__(self, elementsize=4):
        self.elementsize = int(elementsize)

    def decode(self, buf):
        return unshuffle(buf, self.elementsize)


# ----------------------------------------------------------------------------
# storage.py restatement
# ----------------------------------------------------------------------------
def read_block(fh, offset, size):
    """``storage.py:156-162``: positioned read that restores the file cursor."""
    keep = fh.tell()
    fh.seek(offset)
    data = fh.read(size)
    fh.seek(keep)
    return data


def filter_pipeline(chunk, compression, filters):
    """``storage.py:107-123``: undo compression first, then filters in reverse."""
    if compression is not None:
        chunk = compression.decode(chunk)
    for codec in reversed(list(filters or [])):
        chunk = codec.decode(chunk)
    return chunk


def _as_u8(buf):
    # numcodecs.compat.ensure_ndarray (storage.py:57): zero-copy uint8 view
    if isinstance(buf, np.ndarray):
        return buf.view(np.uint8).reshape(-1)
    return np.frombuffer(memoryview(buf), dtype=np.uint8)


def decode_chunk(raw, compression, filters, dtype, shape, order):
    """``storage.py:55-62``: filters, view as ``dtype``, reshape to chunk shape."""
    u8 = _as_u8(filter_pipeline(raw, compression, filters))
    arr = u8.view(dtype)
    return arr.reshape(-1, order="A").reshape(shape, order=order)


def _is_vector(value):
    # storage.py:133,139: lists and ndarrays take the broadcast-equality branch
    return isinstance(value, (list, np.ndarray))


def mask_missing(data, missing):
    """``storage.py:126-153``: union of the four netCDF masking rules.

    Order of the tuple is ``(_FillValue, missing_value, valid_min, valid_max)``
    (``storage.py:130``).  Vector fill/missing values compare element-wise
    with broadcasting (``tests/unit/test_storage.py:9-67``); a non-broadcastable
    missing_value raises ``ValueError`` with the reference's message.
    """
    fill, miss, vmin, vmax = missing
    if fill is not None:
        data = (np.ma.masked_where(data == fill, data) if _is_vector(fill)
                else np.ma.masked_equal(data, fill))
    if miss is not None:
        if _is_vector(miss):
            try:
                data = np.ma.masked_where(data == miss, data)
            except ValueError:
                raise ValueError(
                    "Data and missing_value arrays are not brodcastable!")
        else:
            data = np.ma.masked_equal(data, miss)
    if vmax is not None:
        data = np.ma.masked_greater(data, vmax)
    if vmin is not None:
        data = np.ma.masked_less(data, vmin)
    return data


def _reduce_selected(chunk, chunk_selection, missing, axis, method):
    """``storage.py:95-104``: select, mask, then count + ``method``."""
    sub = mask_missing(chunk[chunk_selection], missing)
    if not method:
        return sub, None
    n = np.ma.count(sub, axis=axis, keepdims=True)
    return method(sub, axis=axis, keepdims=True), n


def reduce_chunk(rfile, offset, size, compression, filters, missing, dtype,
                 shape, order, chunk_selection, axis, method=None,
                 option_disable_chunk_cache=False):
    """``storage.py:8-104`` local-file branch (per-chunk ``print`` dropped)."""
    with open(rfile, "rb") as fh:
        raw = read_block(fh, offset, size)
    chunk = decode_chunk(raw, compression, filters, dtype, shape, order)
    return _reduce_selected(chunk, chunk_selection, missing, axis, method)


def reduce_chunk_bytes(raw, compression, filters, missing, dtype, shape, order,
                       chunk_selection, axis, method=None):
    """Same as :func:`reduce_chunk` for bytes already in memory
    (``storage.py:88-104``, the ``pyfive.high_level.Dataset`` branch)."""
    chunk = decode_chunk(raw, compression, filters, dtype, shape, order)
    return _reduce_selected(chunk, chunk_selection, missing, axis, method)


# ----------------------------------------------------------------------------
# active.py _from_storage combine restatement
# ----------------------------------------------------------------------------
def combine_partials(parts, out_shape, out_dtype, axis, method_name,
                     components=False, order="C"):
    """Restates ``Active._from_storage`` (``active.py:487-516,575-630``).

    ``parts`` is an iterable of ``(tmp, count, out_selection)`` where
    ``out_selection`` already has the reduced axes replaced by the chunk
    coordinate (``active.py:794-799``).  ``out_shape`` is the indexer shape
    with reduced axes replaced by the number of chunks along them
    (``active.py:502-510``).
    """
    fn = {"min": np.ma.min, "max": np.ma.max, "sum": np.ma.sum,
          "mean": np.ma.sum}[method_name]
    need_counts = components or method_name == "mean"
    out = np.ma.empty(out_shape, dtype=out_dtype, order=order)
    out.mask = True
    if need_counts:
        counts = np.ma.empty(out_shape, dtype="int64", order=order)
        counts.mask = True
    for tmp, cnt, sel in parts:
        out[sel] = tmp
        if need_counts:
            counts[sel] = cnt
    out = fn(out, axis=axis, keepdims=True)
    n = np.ma.sum(counts, axis=axis, keepdims=True) if need_counts else None
    if components:
        key = "sum" if method_name == "mean" else method_name
        return {key: out, "n": n}
    if method_name == "mean":
        return out / n
    return out
