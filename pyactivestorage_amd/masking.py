"""Compile ``mask_missing``'s 4-tuple into device thresholds (``pyas_mask``).

Reference: ``activestorage/storage.py:126-153``.  The reference masks with
NumPy comparisons in the *promoted* dtype: e.g. a float32 chunk against a
float64 (or Python float) ``valid_max`` compares in float64, so
``f32(1e20) == 1e20`` is False and ``f32(0.1) > 0.1`` is True.  The device
compares in the storage dtype only, so for every rule the host finds the
exact set of storage-dtype values NumPy would mask and expresses it as a
threshold of that dtype:

* equality  (``masked_equal`` / broadcast ``==``): an interval ``[lo, hi]``
  (conversion to the promoted type is monotone, so the set of values equal to
  ``v`` after promotion is an interval; empty when ``v`` is unrepresentable);
* ``masked_greater(v)``: ``x > t`` with ``t`` the largest value NumPy keeps;
* ``masked_less(v)``:    ``x < u`` with ``u`` the smallest value NumPy keeps.

Each boundary is found by binary search over the ordered values of the
storage dtype using NumPy's own comparison on a one-element probe array of
that dtype as the predicate, so the device reproduces NumPy bit-for-bit
(NaN never masked, ±0 equal, out-of-range and non-representable thresholds,
NEP-50 weak Python scalars, integer/float cross-kind promotion).
"""
from __future__ import annotations

import math
import threading

import numpy as np

from . import _lib
from .dtypes import native, set_scalar

# ---------------------------------------------------------------------------
# ordered value space of a dtype
# ---------------------------------------------------------------------------


class _Space:
    """Bijection between an integer key range and the non-NaN values of dt,
    order-preserving (``-0.0`` and ``+0.0`` get adjacent keys)."""

    def __init__(self, dt):
        self.dt = np.dtype(dt)
        nd = native(dt)
        if nd.kind in "iu":
            info = np.iinfo(nd)
            self.lo, self.hi = int(info.min), int(info.max)
            self.kind = "int"
        else:
            self.bits = nd.itemsize * 8
            self.utype = np.dtype(f"u{nd.itemsize}")
            self.kind = "float"
            self.lo = self._key_of(-np.inf)
            self.hi = self._key_of(np.inf)

    def _key_of(self, v):
        nd = native(self.dt)
        u = int(np.array([v], dtype=nd).view(self.utype)[0])
        sign = 1 << (self.bits - 1)
        return (u | sign) if not (u & sign) else (~u) & ((1 << self.bits) - 1)

    def value(self, key):
        """numpy scalar (native dtype) for key."""
        nd = native(self.dt)
        if self.kind == "int":
            return nd.type(key)
        sign = 1 << (self.bits - 1)
        u = (key & ~sign) if (key & sign) else (~key) & ((1 << self.bits) - 1)
        return np.array([u], dtype=self.utype).view(nd)[0]

    def probe(self, key):
        """One-element array of the *storage* dtype (byte order kept)."""
        return np.array([self.value(key)], dtype=self.dt)


def _first_true(space, pred):
    """Smallest key with pred True for a monotone False..True predicate;
    space.hi + 1 if none."""
    lo, hi = space.lo, space.hi + 1
    while lo < hi:
        mid = (lo + hi) // 2
        if pred(space.probe(mid)):
            hi = mid
        else:
            lo = mid + 1
    return lo


def _bool(mask_or_values):
    """First element of a boolean (mask) array as a Python bool."""
    return bool(np.asarray(mask_or_values)[0])


def _val(x):
    """First element of a comparison result (MaskedArray or ndarray)."""
    if isinstance(x, np.ma.MaskedArray):
        x = x.filled(False)
    return bool(np.asarray(x)[0])


# ---------------------------------------------------------------------------
# rule compilers; each returns ("none" | "all" | "set", payload)
# ---------------------------------------------------------------------------


def _quiet(fn):
    def wrapped(*a):
        with np.errstate(all="ignore"):
            return fn(*a)
    return wrapped


def _gt_rule(space, value):
    """masked_greater(data, value): mask x > t  (storage.py:145-146)."""
    pred = _quiet(lambda p: _bool(np.ma.getmaskarray(np.ma.masked_greater(p, value))))
    k = _first_true(space, pred)
    if k > space.hi:
        return ("none", None)
    if k == space.lo:
        return ("all", None)
    return ("set", space.value(k - 1))


def _lt_rule(space, value):
    """masked_less(data, value): mask x < u  (storage.py:148-149)."""
    pred = _quiet(lambda p: not _bool(np.ma.getmaskarray(np.ma.masked_less(p, value))))
    k = _first_true(space, pred)  # first value NOT masked
    if k > space.hi:
        return ("all", None)
    if k == space.lo:
        return ("none", None)
    return ("set", space.value(k))


def _eq_interval(space, eq, less, greater):
    """Interval of values x with eq(x) given monotone less/greater predicates
    of the same promotion.  Returns (lo, hi) numpy scalars or None."""
    k_lo = _first_true(space, lambda p: not less(p))       # first x with not (x < v)
    k_hi = _first_true(space, lambda p: greater(p)) - 1    # last x with not (x > v)
    if k_lo > k_hi:
        return None
    if not (eq(space.probe(k_lo)) and eq(space.probe(k_hi))):
        return None
    return (space.value(k_lo), space.value(k_hi))


def _eq_scalar(space, value):
    """masked_equal(data, value) (storage.py:136,144)."""
    eq = _quiet(lambda p: _bool(np.ma.getmaskarray(np.ma.masked_equal(p, value))))
    eq(space.probe(space.lo))  # raise masked_equal's own errors first (fill_value setter)
    less = _quiet(lambda p: _val(np.ma.less(p, value)))
    greater = _quiet(lambda p: _val(np.ma.greater(p, value)))
    return _eq_interval(space, eq, less, greater)


def _eq_element(space, elem):
    """Broadcast ``data == vector`` (storage.py:133-134,139-141) for one
    element of the vector, kept as a 1-element array of the vector's dtype."""
    eq = _quiet(lambda p: bool(np.asarray(p == elem)[0]))
    less = _quiet(lambda p: bool(np.asarray(p < elem)[0]))
    greater = _quiet(lambda p: bool(np.asarray(p > elem)[0]))
    return _eq_interval(space, eq, less, greater)


# ---------------------------------------------------------------------------
# public API
# ---------------------------------------------------------------------------


def _is_vector(v):
    return isinstance(v, (list, np.ndarray))


def _key(v):
    """Hashable, type-faithful cache key for a missing attribute."""
    if v is None:
        return None
    if _is_vector(v):
        a = np.asarray(v)
        return ("vec", type(v).__name__, a.dtype.str, a.shape, a.tobytes())
    if isinstance(v, np.generic):
        return ("np", np.dtype(type(v)).str, np.asarray(v).tobytes())
    if isinstance(v, float) and math.isnan(v):
        return ("py", "float", "nan")
    return ("py", type(v).__name__, v)


class CompiledMask:
    """Device-ready form of one missing 4-tuple for one storage dtype.

    ``tables`` holds host arrays (lo, hi, strides) for vector
    fill/missing values; they are uploaded per call by the caller.
    """

    def __init__(self, dt):
        self.dt = np.dtype(dt)
        self.flags = 0
        self.eq = [None, None]          # (lo, hi) numpy scalars
        self.gt = None
        self.lt = None
        self.vectors = [None, None]     # np arrays of the raw vector values
        self.tables = [None, None]      # (lo array, hi array, valid bool array)
        self.any_rule = False           # a masking attribute was given at all

    @property
    def masked(self) -> bool:
        """True when the reference would return a MaskedArray (any attr set)."""
        return self.any_rule

    def to_struct(self, sel_shape=None, table_ptrs=None):
        """Fill a ``_lib.Mask``.  For vector rules ``table_ptrs[k]`` gives the
        device pointers (lo, hi) and ``sel_shape`` the selected array shape."""
        m = _lib.Mask()
        m.flags = self.flags
        nd = native(self.dt)
        for k in range(2):
            if self.eq[k] is not None:
                set_scalar(m.eq_lo[k], self.eq[k][0], nd)
                set_scalar(m.eq_hi[k], self.eq[k][1], nd)
        if self.gt is not None:
            set_scalar(m.gt, self.gt, nd)
        if self.lt is not None:
            set_scalar(m.lt, self.lt, nd)
        return m


_cache: dict = {}
_cache_lock = threading.Lock()
_CACHE_CAP = 512   # compiled masks kept; keys can come from clients (reductionist_server)


def compile_missing(missing, dt) -> CompiledMask:
    """Compile ``(fill_value, missing_value, valid_min, valid_max)``."""
    if missing is None:
        missing = (None, None, None, None)
    fill, miss, vmin, vmax = missing
    dt = np.dtype(dt)
    key = (dt.str, _key(fill), _key(miss), _key(vmin), _key(vmax))
    hit = _cache.get(key)
    if hit is not None:
        return hit
    space = _Space(dt)
    cm = CompiledMask(dt)
    info_min = space.value(space.lo)
    info_max = space.value(space.hi)
    all_masked = False
    for k, (val, bit) in enumerate(((fill, _lib.MASK_EQ0), (miss, _lib.MASK_EQ1))):
        if val is None:
            continue
        cm.any_rule = True
        if _is_vector(val):
            arr = np.asarray(val)
            cm.vectors[k] = arr
            flat = arr.reshape(-1)
            if flat.size == 1:
                iv = _eq_element(space, flat[0:1])
                if iv is not None:
                    cm.eq[k] = iv
                    cm.flags |= bit
            else:
                los, his, ok = [], [], []
                for i in range(flat.size):
                    iv = _eq_element(space, flat[i:i + 1])
                    if iv is None:
                        los.append(info_max); his.append(info_min); ok.append(False)
                    else:
                        los.append(iv[0]); his.append(iv[1]); ok.append(True)
                cm.tables[k] = (np.array(los, dtype=native(dt)), np.array(his, dtype=native(dt)),
                                np.array(ok, dtype=bool))
                cm.flags |= _lib.MASK_TAB0 if k == 0 else _lib.MASK_TAB1
        else:
            iv = _eq_scalar(space, val)
            if iv is not None:
                cm.eq[k] = iv
                cm.flags |= bit
    if vmax is not None:
        cm.any_rule = True
        kind, t = _gt_rule(space, vmax)
        if kind == "set":
            cm.gt = t
            cm.flags |= _lib.MASK_GT
        elif kind == "all":
            all_masked = True
    if vmin is not None:
        cm.any_rule = True
        kind, u = _lt_rule(space, vmin)
        if kind == "set":
            cm.lt = u
            cm.flags |= _lib.MASK_LT
        elif kind == "all":
            all_masked = True
    if all_masked:
        # Only integer dtypes can have every value masked (float NaN never is).
        # x > MIN masks all but MIN; x < MIN+1 masks MIN.
        cm.gt = info_min
        cm.flags |= _lib.MASK_GT
        nxt = space.value(space.lo + 1)
        cm.lt = nxt if cm.lt is None or cm.lt < nxt else cm.lt
        cm.flags |= _lib.MASK_LT
    with _cache_lock:   # callers: the 30-thread drop-in pool, Reductionist request threads
        while len(_cache) >= _CACHE_CAP:
            _cache.pop(next(iter(_cache)))   # oldest first (dicts keep insertion order)
        _cache[key] = cm
    return cm


def table_layout(cm: CompiledMask, k: int, sel_shape, which: str):
    """Broadcast strides (in table elements) of vector rule k over the selected
    array shape, replicating the reference's errors (storage.py:139-143 and
    numpy.ma.masked_where's shape check)."""
    arr = cm.vectors[k]
    try:
        out_shape = np.broadcast_shapes(tuple(sel_shape), arr.shape)
    except ValueError:
        if which == "missing_value":
            raise ValueError("Data and missing_value arrays are not brodcastable!") from None
        raise ValueError(f"operands could not be broadcast together with shapes "
                         f"{tuple(sel_shape)} {arr.shape}") from None
    if tuple(out_shape) != tuple(sel_shape):
        raise IndexError("Inconsistent shape between the condition and the input "
                         f"(got {tuple(out_shape)} and {tuple(sel_shape)})")
    idx = np.broadcast_to(np.arange(arr.size, dtype=np.int64).reshape(arr.shape), tuple(sel_shape))
    return [s // 8 for s in idx.strides]
