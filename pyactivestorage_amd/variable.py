"""Variable metadata the planner needs: what pyfive gives the reference.

``ChunkedVariable`` carries shape, chunk shape, dtype, the HDF5 filter
pipeline, the masking attributes and the chunk index (chunk coordinates ->
byte offset and size; ``ds.get_chunk_info_from_chunk_coord`` at
``activestorage/active.py:663-665``).  Chunk bytes come from a reader
callable, by default a positioned read of the file (``storage.py:156-162``).

``get_missing_attributes`` restates ``active.py:126-159`` and
``decode_filters`` restates ``hdf2numcodec.py:4-89`` (without its
``compressors[0]`` IndexError on shuffle-only pipelines).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from .storage import Shuffle, Zlib

GZIP_DEFLATE_FILTER = 1   # hdf2numcodec.py:94-97 (pyfive's HDF5 filter ids)
SHUFFLE_FILTER = 2


def get_missing_attributes(attrs) -> tuple:
    """``(_FillValue, missing_value, valid_min, valid_max)`` from variable
    attributes, as ``active.py:126-159`` builds it."""

    def one(x):  # hfix: unwrap single-element lists/arrays (active.py:131-140)
        if x is None:
            return x
        if not np.isscalar(x) and len(x) == 1:
            return x[0]
        return x

    fill = one(attrs.get("_FillValue"))
    missing = attrs.get("missing_value")
    if isinstance(missing, np.ndarray) and missing.size == 1:   # active.py:145-147
        missing = missing[0]
    vmin = one(attrs.get("valid_min"))
    vmax = one(attrs.get("valid_max"))
    vrange = one(attrs.get("valid_range"))
    if vmax is not None or vmin is not None:
        if vrange is not None:
            raise ValueError("Invalid combination in the file of valid_min, valid_max, "
                             f"valid_range: {vmin}, {vmax}, {vrange}")
    elif vrange is not None:
        vmin, vmax = vrange
    return fill, missing, vmin, vmax


def decode_filters(filter_pipeline, itemsize, name):
    """HDF5 filter pipeline -> (compressor, filters) (``hdf2numcodec.py:4-89``).

    Deflate (id 1) -> Zlib(level); shuffle (id 2) -> Shuffle(itemsize); any
    other id -> NotImplementedError; two compressors -> ValueError."""
    compressors, filters = [], []
    for f in filter_pipeline or []:
        fid = f["filter_id"]
        props = f.get("client_data", ())
        if fid == GZIP_DEFLATE_FILTER:
            compressors.append(Zlib(level=props[0] if len(props) else 1))
        elif fid == SHUFFLE_FILTER:
            filters.append(Shuffle(elementsize=itemsize))
        else:
            raise NotImplementedError("We cannot yet support filter id ", fid)
    if len(compressors) > 1:
        raise ValueError("We only expected one compression algorithm")
    return (compressors[0] if compressors else None), filters


@dataclass
class ChunkedVariable:
    """One netCDF4/HDF5 variable as the planner sees it."""
    name: str
    shape: tuple
    chunks: tuple
    dtype: np.dtype
    chunk_index: dict                      # coords tuple -> (byte offset, size)
    attrs: dict = field(default_factory=dict)
    filter_pipeline: Optional[list] = None  # [{"filter_id": int, "client_data": [...]}]
    order: str = "C"
    filename: Optional[str] = None
    reader: Optional[Callable[[int, int], bytes]] = None   # (offset, size) -> bytes

    def __post_init__(self):
        self.shape = tuple(int(s) for s in self.shape)
        self.chunks = tuple(int(c) for c in self.chunks)
        self.dtype = np.dtype(self.dtype)
        if len(self.chunks) != len(self.shape):
            raise ValueError("chunk rank differs from variable rank")

    @property
    def ndim(self):
        return len(self.shape)

    def read(self, offset, size) -> bytes:
        if self.reader is not None:
            return self.reader(offset, size)
        with open(self.filename, "rb") as fh:
            return os.pread(fh.fileno(), size, offset)

    def chunk_info(self, coords):
        try:
            return self.chunk_index[tuple(int(c) for c in coords)]
        except KeyError:
            raise KeyError(f"chunk {tuple(coords)} of {self.name} is not allocated") from None
