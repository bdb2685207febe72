"""NumPy dtype <-> pyas dtype codes, and the result-dtype rules of the
reference's reductions (``storage.py:98-100`` with ``np.ma.*`` methods, and
``active.py:512,630`` for the combine)."""
from __future__ import annotations

import numpy as np

from . import _lib

_CODES = {
    ("i", 1): _lib.I8, ("u", 1): _lib.U8, ("i", 2): _lib.I16, ("u", 2): _lib.U16,
    ("i", 4): _lib.I32, ("u", 4): _lib.U32, ("i", 8): _lib.I64, ("u", 8): _lib.U64,
    ("f", 4): _lib.F32, ("f", 8): _lib.F64,
}


def dtype_code(dt) -> int:
    dt = np.dtype(dt)
    try:
        return _CODES[(dt.kind, dt.itemsize)]
    except KeyError:
        raise NotImplementedError(f"dtype {dt} is not a netCDF-4 numeric type") from None


def needs_byteswap(dt) -> bool:
    dt = np.dtype(dt)
    return dt.itemsize > 1 and not dt.isnative


def native(dt) -> np.dtype:
    return np.dtype(dt).newbyteorder("=")


def value_class(dt) -> str:
    """Which member of pyas_scalar carries values of this dtype."""
    k = np.dtype(dt).kind
    return {"f": "f", "i": "i", "u": "u"}[k]


def sum_dtype(dt) -> np.dtype:
    """``np.ma.sum`` result dtype: floats keep theirs, ints widen to 64 bit."""
    dt = native(dt)
    if dt.kind == "i":
        return np.dtype(np.int64)
    if dt.kind == "u":
        return np.dtype(np.uint64)
    return dt


def mean_dtype(dt, masked: bool) -> np.dtype:
    """Result dtype of ``np.ma.mean``/``np.mean`` on the selected chunk.

    Masked arrays take MaskedArray.mean (``dsum * 1. / cnt`` -> float64);
    unmasked ones take ndarray.mean (floats keep their dtype, ints -> f64).
    """
    dt = native(dt)
    if masked or dt.kind in "iu":
        return np.dtype(np.float64)
    return dt


def scalar_value(s, dt):
    """Extract a pyas_scalar as a numpy scalar of (native) dtype ``dt``."""
    dt = native(dt)
    if dt.kind == "f":
        return dt.type(s.f)
    if dt.kind == "i":
        return np.int64(s.i).astype(dt)
    return np.uint64(s.u).astype(dt)


def set_scalar(s, value, dt) -> None:
    dt = native(dt)
    if dt.kind == "f":
        s.f = float(value)
    elif dt.kind == "i":
        s.i = int(value)
    else:
        s.u = int(value)
