"""Turn device partials into exactly the objects the reference returns.

``storage.reduce_chunk`` returns ``(method(tmp, axis, keepdims=True),
np.ma.count(tmp, axis, keepdims=True))`` (``storage.py:98-100``).  The
container and dtype depend on the method and on whether ``mask_missing``
produced a MaskedArray (any masking attribute present, ``storage.py:130-153``):

* ``np.ma.sum/min/max/mean`` -> MaskedArray (mask ``nomask`` when unmasked,
  a full boolean mask when masked);
* ``np.sum/min/max/mean``    -> plain ndarray when unmasked, MaskedArray when
  masked (NumPy dispatches to the MaskedArray methods);
* sum widens ints to int64/uint64; min/max keep the dtype; mean is float64
  for masked data and ints, and keeps float32 for unmasked float32
  (ndarray.mean).  Byte order of results is native, as NumPy's.
"""
from __future__ import annotations

import numpy as np

from .dtypes import mean_dtype, native, sum_dtype

_METHODS = {}
METHODS = _METHODS   # callable -> (kind, is_ma), for hot-path lookups


def _register():
    for fn, kind, ma in (
        (np.ma.sum, "sum", True), (np.sum, "sum", False),
        (np.ma.min, "min", True), (np.min, "min", False), (np.amin, "min", False),
        (np.ma.max, "max", True), (np.max, "max", False), (np.amax, "max", False),
        (np.ma.mean, "mean", True), (np.mean, "mean", False),
    ):
        _METHODS.setdefault(fn, (kind, ma))


_register()


def method_kind(method):
    """(kind, is_ma) for a reduction callable or a controlled-vocabulary name."""
    if isinstance(method, str):
        if method not in ("sum", "min", "max", "mean"):
            raise ValueError(f"Bad 'method': {method}. Choose from min/max/mean/sum.")
        return method, True
    try:
        return _METHODS[method]
    except (KeyError, TypeError):
        raise NotImplementedError(
            f"reduction method {method!r} is not supported by the MI355X backend "
            "(supported: sum, min, max, mean from numpy / numpy.ma)") from None


def _no_identity(kind):
    name = {"min": "minimum", "max": "maximum"}[kind]
    return ValueError(f"zero-size array to reduction operation {name} which has no identity")


def build(parts: np.ndarray, kind: str, is_ma: bool, dt, has_rule: bool, n_reduced: int,
          n_selected: int):
    """``parts``: structured partials already shaped like the keepdims result.

    ``has_rule``: a masking attribute was given (mask_missing returned a
    MaskedArray).  NumPy shrinks an all-False mask to ``nomask``
    (numpy.ma.masked_where -> _shrink_mask), so the result only carries a
    mask array when some selected element was actually masked.
    """
    dt = np.dtype(dt)
    nd = native(dt)
    count = np.ascontiguousarray(parts["count"]).astype(np.int64)
    any_masked = has_rule and int(count.sum()) < n_selected
    if kind == "sum":
        vals = parts["sum"].astype(sum_dtype(dt))
    elif kind in ("min", "max"):
        if n_reduced == 0:
            raise _no_identity(kind)
        vals = parts[kind].astype(nd)
    else:  # mean
        s = parts["sum"].astype(sum_dtype(dt))
        with np.errstate(divide="ignore", invalid="ignore"):
            if any_masked:
                # MaskedArray.mean: dsum * 1. / cnt  (float64 result)
                vals = (s * 1.0) / count
            elif nd.kind in "iu":
                vals = s.astype(np.float64) / np.float64(n_reduced if n_reduced else np.nan)
            else:
                # ndarray.mean: ret.dtype.type(ret / rcount) keeps float32
                vals = (s / nd.type(n_reduced)).astype(nd) if n_reduced else s.astype(nd) * np.nan
        vals = np.asarray(vals, dtype=mean_dtype(dt, any_masked))
    vals = np.ascontiguousarray(vals)
    if any_masked:
        mask = count == 0
        if kind == "mean":
            # np.ma true_divide is a domained op: non-finite quotients are masked
            mask = mask | ~np.isfinite(vals)
        return np.ma.MaskedArray(vals, mask=mask), count
    if has_rule or is_ma:
        return np.ma.MaskedArray(vals), count
    return vals, count


def _ma(vals, mask=None):
    """``np.ma.MaskedArray(vals[, mask=mask])`` without the constructor's
    argument handling: a view with the constructor's exact attribute state
    (``_mask`` the given array or nomask, ``_sharedmask`` True)."""
    r = vals.view(np.ma.MaskedArray)
    if mask is not None:
        r._mask = mask
    r._sharedmask = True
    return r


def build_one(p, shape, kind: str, is_ma: bool, dt, has_rule: bool, n_reduced: int,
              n_selected: int):
    """:func:`build` for ONE partial ``p`` (a structured scalar), i.e. every
    selected dim reduced: the same objects with a fraction of the overhead
    (the per-chunk drop-in's common case, storage.py:98-100 with the full
    axis tuple)."""
    if kind == "mean" or (kind != "sum" and n_reduced == 0):
        return build(np.array(p).reshape(shape), kind, is_ma, dt, has_rule, n_reduced, n_selected)
    cnt = int(p["count"])
    count = np.array(cnt, dtype=np.int64).reshape(shape)
    if kind == "sum":
        vals = np.array(p["sum"], dtype=sum_dtype(dt)).reshape(shape)
    else:
        vals = np.array(p[kind], dtype=native(dt)).reshape(shape)
    if has_rule and cnt < n_selected:
        return _ma(vals, np.array(cnt == 0).reshape(shape)), count
    if has_rule or is_ma:
        return _ma(vals), count
    return vals, count
