"""NumPy's sign of a zero min/max, as a rule the device can apply.

``storage.py:99-100`` returns ``np.ma.min/max(chunk, axis, keepdims=True)``.
When the extreme value is zero and the data hold both ``+0.0`` and
``-0.0``, which zero NumPy returns depends on how its reduction loop visits
the elements: the loop (``numpy/_core/src/umath/loops_minmax``, contiguous
reduce) keeps one accumulator per SIMD lane initialised with the running
result, lets a later element win a tie inside its lane, folds the lanes in a
fixed tree (ties go one way per tree level), then runs the scalar remainder
(later elements win); the iterator hands it the flattened C-ordered data in
pieces of ``np.getbufsize()`` elements, the first piece starting after the
element that seeds the result.

The lane count and the lane tree depend on the SIMD target NumPy dispatches
on the host CPU (AVX512: 16 float32 / 8 float64 lanes; AVX2 has fewer), so
the rule is not hard-coded: :func:`tie_rule` derives it from NumPy itself
on this host (a few tiny ``np.min`` calls) and checks it on random data
before the device uses it.  The device then reproduces the sign per chunk
(``pyas_zero_sign_chunks``) and across the chunk sequence
(``pyas_zero_sign_seq``):``tests/test_zero_sign.py`` pins the derived
rule against NumPy and ``tests/test_gpu_zero_sign.py`` the device result.
"""
from __future__ import annotations

import threading

import numpy as np

_LOCK = threading.Lock()
_RULES: dict = {}


def _derive(dt: np.dtype, lanes: int):
    """Lane priority under the assumption of `lanes` lanes: lane order in
    which a lone -0.0 in one vector (all else +0.0 or larger) decides."""
    n = 1 + lanes
    order, excluded = [], []
    for _ in range(lanes):
        found = None
        for lane in range(lanes):
            if lane in excluded:
                continue
            a = np.zeros(n, dt)
            a[0] = 1.0
            for e in excluded:
                a[1 + e] = 1.0
            a[1 + lane] = -0.0
            if np.signbit(np.min(a)):
                found = lane
                break
        if found is None:
            return None
        order.append(found)
        excluded.append(found)
    return order


def emulate(a: np.ndarray, op, lanes: int, order, piece: int):
    """Sign bit NumPy's contiguous reduce gives ``op`` (np.min / np.max)
    over the flattened C-ordered ``a`` when the result is zero, else None.
    Python restatement of the rule the device applies (checking only)."""
    a = np.ascontiguousarray(a).reshape(-1)
    if a.size == 0:
        return None
    vals = a if op is np.min else -a
    r = (vals[0], bool(np.signbit(a[0])))
    bounds = sorted(set([1] + list(range(piece, a.size, piece)) + [a.size]))
    for s, e in zip(bounds[:-1], bounds[1:]):
        seg, raw = vals[s:e], a[s:e]
        m = e - s
        nv = m - m % lanes
        lane_v = [r] * lanes
        for lane in range(lanes):
            idx = np.arange(lane, nv, lanes)
            if idx.size == 0:
                continue
            mn = seg[idx].min()
            if mn <= lane_v[lane][0]:
                last = idx[np.flatnonzero(seg[idx] == mn)[-1]]
                lane_v[lane] = (mn, bool(np.signbit(raw[last])))
        best = min(v[0] for v in lane_v)
        for lane in order:
            if lane_v[lane][0] == best:
                r = lane_v[lane]
                break
        for i in range(nv, m):
            if seg[i] <= r[0]:
                r = (seg[i], bool(np.signbit(raw[i])))
    return r[1] if r[0] == 0 else None


def _validate(dt, lanes, order, piece) -> bool:
    rng = np.random.default_rng(1234)
    for trial in range(48):
        n = int(rng.integers(2, 200)) if trial % 2 else int(rng.integers(200, 3 * piece))
        for op, sgn in ((np.min, 1.0), (np.max, -1.0)):
            a = (rng.uniform(0.5, 2.0, n) * sgn).astype(dt)
            k = int(rng.integers(1, 6))
            pos = rng.integers(0, n, k)
            a[pos] = np.where(rng.random(k) < 0.5, -0.0, 0.0)
            want = bool(np.signbit(op(a)))
            if emulate(a, op, lanes, order, piece) != want:
                return False
    return True


class TieRule:
    """lanes, lane priority (``order``: lanes from highest priority; ``rank``
    = position of each lane in it) and piece size of NumPy's reduce loop."""

    def __init__(self, lanes, order, piece):
        self.lanes = int(lanes)
        self.order = list(order)
        self.rank = [0] * self.lanes
        for r, lane in enumerate(self.order):
            self.rank[lane] = r
        self.piece = int(piece)


def tie_rule(dtype):
    """The validated :class:`TieRule` of float32 or float64 on this host, or
    None when no candidate rule reproduces NumPy (the device then leaves the
    sign as its own reduction produced it)."""
    dt = np.dtype(dtype).newbyteorder("=")
    if dt.kind != "f" or dt.itemsize not in (4, 8):
        return None
    with _LOCK:
        if dt.str in _RULES:
            return _RULES[dt.str]
        piece = int(np.getbufsize())
        rule = None
        for lanes in (16, 8, 32, 4, 64, 2, 1):
            order = _derive(dt, lanes)
            if order is not None and _validate(dt, lanes, order, piece):
                rule = TieRule(lanes, order, piece)
                break
        _RULES[dt.str] = rule
        return rule
