"""NumPy's sign of a zero min/max, as a rule the device can apply.

``storage.py:99-100`` returns ``np.ma.min/max(chunk[sel], axis,
keepdims=True)`` and ``active.py:594`` reduces the ``out`` array of
per-chunk results the same way.  When an extreme is zero and its elements
hold both ``+0.0`` and ``-0.0``, which zero NumPy returns depends on the
order its reduction visits the elements.  Measured on NumPy 2.2 (this
module derives the host-dependent parts from NumPy at start-up and checks
them on random data):

* **Iteration.**  The iterator walks the reduced array in memory order (its
  dims sorted by ``|stride|``; C order for C-ordered chunks and slices),
  drops extent-1 dims and coalesces neighbours.  For each output the first
  element in that order seeds the result.  The *trailing group* is the run
  of reduced dims at the inner end of the order.
* **Calls.**  If the innermost dim is kept, the loop is elementwise
  (``out[i] = min(out[i], x[i])``): every element is its own call.
  Otherwise every run of the trailing group is one call of the reduce loop
  (length ``Lr`` = the group's size; a group of several dims that do not
  coalesce is copied to a contiguous buffer first, as is any non-native
  byte order).  Calls are cut into pieces of ``np.getbufsize()`` elements
  from the run's start; the first piece of the first run starts after the
  seed.
* **A contiguous call** (SIMD): one accumulator per lane, seeded with the
  running result, a later element wins a tie in its lane; the lanes are
  folded in a fixed priority order; then the scalar remainder (later wins).
* **A strided call** (a non-contiguous inner dim of a view): ``acc``
  accumulators seeded with the call's first elements, later wins per
  accumulator, folded in a fixed priority order, then merged into the
  running result (the call's zero wins), then the remainder (later wins).

Which zero wins is then a function of the zeros' positions alone, which the
device evaluates with two order-free keys per output (``keys`` below):

* ``K1`` = max over the *significant* zeros of ``(e + 1) << 1 | sign``:
  the seed, zeros in the top-priority lane and remainder zeros;
* ``W`` = min over all zeros of ``(row, lane rank, -offset)``: the winner
  of the first row (call piece) that holds any zero, which decides only
  while no zero is in hand;
* result = the later of the two (a strided call orders its zeros by one
  key ``(call, remainder?, acc priority, offset)`` instead).

Both keys combine by max/min, so the per-chunk pass (``pyas_tie_chunks``),
the pass over the ``out`` grid (``pyas_tie_grid``) and ranks of a
torch.distributed group (keys gathered, then ``pyas_tie_finalize``) use the
same arithmetic.  :func:`predict` restates it over a NumPy array;
``tests/test_zero_sign.py`` checks it against NumPy and
``tests/test_gpu_zero_sign.py`` the device against both.
"""
from __future__ import annotations

import threading

import numpy as np

_LOCK = threading.Lock()
_RULES: dict = {}

GEOM_VIEW = 1        # the reduced array is the chunk[sel] view itself (strides from the selection)
GEOM_BUFFERED = 2    # non-native byte order: every reduce call runs over a contiguous buffer

W_NONE = (1 << 64) - 1
OFF_BITS = 24        # offsets inside a piece (piece <= 2^24 elements)
REM_RANK = 127


def _derive(dt: np.dtype, lanes: int, strided: bool = False):
    """Lane (or accumulator) priority under the assumption of `lanes`:
    the lane order in which a lone -0.0 in one vector (all else +0.0 or
    larger) decides.  ``strided``: through a stride-2 view (the strided
    reduce loop)."""
    n = 1 + lanes
    order, excluded = [], []
    for _ in range(lanes):
        found = None
        for lane in range(lanes):
            if lane in excluded:
                continue
            base = np.zeros(2 * n if strided else n, dt)
            a = base[::2] if strided else base
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


def _lane_call(r, seg, raw, lanes, order):
    """One contiguous reduce call (vals seg, raw values raw) on running r."""
    m = len(seg)
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
    if nv:
        best = min(v[0] for v in lane_v)
        for lane in order:
            if lane_v[lane][0] == best:
                r = lane_v[lane]
                break
    for i in range(nv, m):
        if seg[i] <= r[0]:
            r = (seg[i], bool(np.signbit(raw[i])))
    return r


def _acc_call(r, seg, raw, acc, order):
    """One strided reduce call: accumulators seeded with the first elements."""
    m = len(seg)
    nv = m - m % acc
    if nv:
        accs = [(seg[k], bool(np.signbit(raw[k]))) for k in range(acc)]
        for i in range(acc, nv):
            k = i % acc
            if seg[i] <= accs[k][0]:
                accs[k] = (seg[i], bool(np.signbit(raw[i])))
        best = min(v[0] for v in accs)
        f = next(accs[k] for k in order if accs[k][0] == best)
        if f[0] <= r[0]:
            r = f
    for i in range(nv, m):
        if seg[i] <= r[0]:
            r = (seg[i], bool(np.signbit(raw[i])))
    return r


def emulate(a: np.ndarray, op, lanes: int, order, piece: int):
    """Sign bit NumPy's contiguous reduce gives ``op`` (np.min / np.max)
    over the flattened C-ordered ``a`` when the result is zero, else None.
    Sequential restatement of the loop (checking only)."""
    a = np.ascontiguousarray(a).reshape(-1)
    if a.size == 0:
        return None
    vals = a if op is np.min else -a
    r = (vals[0], bool(np.signbit(a[0])))
    bounds = sorted(set([1] + list(range(piece, a.size, piece)) + [a.size]))
    for s, e in zip(bounds[:-1], bounds[1:]):
        r = _lane_call(r, vals[s:e], a[s:e], lanes, order)
    return r[1] if r[0] == 0 else None


def _emulate_strided(a: np.ndarray, op, acc: int, order, piece: int):
    """The strided loop over a 1-D view (checking only)."""
    vals = a if op is np.min else -a
    r = (vals[0], bool(np.signbit(a[0])))
    bounds = sorted(set([1] + list(range(piece, a.size, piece)) + [a.size]))
    for s, e in zip(bounds[:-1], bounds[1:]):
        r = _acc_call(r, vals[s:e], a[s:e], acc, order)
    return r[1] if r[0] == 0 else None


def _zeros_data(rng, n, dt, op, dense):
    a = (rng.uniform(0.5, 2.0, n) * (1.0 if op is np.min else -1.0)).astype(dt)
    if dense:
        z = rng.random(n) < rng.choice([0.05, 0.3, 0.8])
        a[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
    else:
        k = int(rng.integers(1, 6))
        pos = rng.integers(0, n, k)
        a[pos] = np.where(rng.random(k) < 0.5, -0.0, 0.0)
    return a


def _validate(dt, lanes, order, piece) -> bool:
    rng = np.random.default_rng(1234)
    for trial in range(48):
        n = int(rng.integers(2, 200)) if trial % 2 else int(rng.integers(200, 3 * piece))
        for op in (np.min, np.max):
            a = _zeros_data(rng, n, dt, op, trial % 3 == 0)
            want = bool(np.signbit(op(a)))
            if emulate(a, op, lanes, order, piece) != want:
                return False
    return True


def _validate_acc(dt, acc, order, piece) -> bool:
    rng = np.random.default_rng(4321)
    for trial in range(32):
        n = int(rng.integers(2, 100)) if trial % 2 else int(rng.integers(100, 2 * piece + 50))
        step = int(rng.choice([2, 3, -1, -2]))
        for op in (np.min, np.max):
            base = _zeros_data(rng, n * abs(step), dt, op, trial % 3 == 0)
            v = base[::step][:n]
            if v.size < 2 or op(v) != 0:
                continue
            if _emulate_strided(v, op, acc, order, piece) != bool(np.signbit(op(v))):
                return False
    return True


class TieRule:
    """NumPy's reduce loops on this host: ``lanes`` and lane priority
    (``order``: lanes from highest priority; ``rank`` = position of each lane
    in it) of the contiguous loop, ``acc`` accumulators and their priority of
    the strided loop, and the iterator's piece size."""

    def __init__(self, lanes, order, piece, acc=0, acc_order=()):
        self.lanes = int(lanes)
        self.order = list(order)
        self.rank = [0] * self.lanes
        for r, lane in enumerate(self.order):
            self.rank[lane] = r
        self.piece = int(piece)
        self.acc = int(acc)
        self.acc_order = list(acc_order)
        self.acc_rank = [0] * self.acc
        for r, k in enumerate(self.acc_order):
            self.acc_rank[k] = r


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
        if piece < (1 << OFF_BITS):
            for lanes in (16, 8, 32, 4, 64, 2, 1):
                order = _derive(dt, lanes)
                if order is not None and _validate(dt, lanes, order, piece):
                    for acc in (8, 4, 16, 2, 1):
                        ao = _derive(dt, acc, strided=True)
                        if ao is not None and _validate_acc(dt, acc, ao, piece):
                            rule = TieRule(lanes, order, piece, acc, ao)
                            break
                    break
        _RULES[dt.str] = rule
        return rule


# ---------------------------------------------------------------------------
# the device's algorithm, restated over a NumPy array (tests check it against
# NumPy itself; pyas_kernels.hpp tie_* implements it)
# ---------------------------------------------------------------------------
MODE_LANES, MODE_ACC = 0, 1


def call_structure(counts, strides, reduced, perm, buffered, piece=None):
    """Reduce calls of one reduction: ``counts``/``strides`` (elements) of
    the reduced array per dim, ``reduced`` a set of dims, ``perm`` the
    iteration order (outer -> inner).  Returns ``(mode, Lr, n_copy,
    block)``: Lr = 1 for elementwise calls; in MODE_ACC the first
    ``n_copy`` runs of the iteration are nevertheless contiguous calls
    (NumPy's first buffer fill spans more than one kept dim and is copied),
    ``block`` = the kept dims of that first fill, inner first."""
    inner = [d for d in perm if counts[d] != 1]
    group = []
    for d in reversed(inner):
        if d not in reduced:
            break
        group.append(d)               # innermost first
    if not group:
        return MODE_LANES, 1, 0, []
    lr = 1
    for d in group:
        lr *= counts[d]
    one_dim = all(strides[o] == strides[i] * counts[i] for i, o in zip(group, group[1:]))
    if not one_dim or buffered or strides[group[0]] == 1:
        return MODE_LANES, lr, 0, []
    # the kept iteration dims right outside the group, up to a reduced one
    rest = list(reversed(inner))[len(group):]
    block = []
    for d in rest:
        if d in reduced:
            break
        block.append(d)
    n_copy = 0
    if block and piece:
        first = counts[block[0]]      # the first kept iteration dim (coalesced)
        for i, o in zip(block, block[1:]):
            if strides[o] != strides[i] * counts[i]:
                break
            first *= counts[o]
        kb = 1
        for d in block:
            kb *= counts[d]
        n1 = min(piece // lr, kb)
        if n1 > first:
            n_copy = n1
    return MODE_ACC, lr, n_copy, block


def element_keys(e, sign, mode, lr, rule, lanes=None):
    """(K1, W, KA) keys of zero elements at reduced positions e (int64
    array) with sign bits ``sign`` (0/1 array).  ``lanes``: in MODE_ACC,
    which elements sit in a contiguous (copied) call."""
    e = np.asarray(e, dtype=np.int64)
    s = np.asarray(sign, dtype=np.uint64)
    P = rule.piece
    npr = (lr + P - 1) // P
    q, pos = e // lr, e % lr
    k = pos // P
    s0 = np.where((q == 0) & (k == 0), 1, k * P)
    e1 = np.minimum((k + 1) * P, lr)
    m = e1 - s0
    off = pos - s0
    row = q * npr + k
    seed = e == 0
    none = np.zeros(e.shape, dtype=np.uint64)
    ka = none
    if mode == MODE_ACC:
        acc = rule.acc
        nv = m - m % acc
        vec = off < nv
        prio = np.where(vec, acc - 1 - np.array(rule.acc_rank, dtype=np.int64)[np.where(vec, off % acc, 0)], 0)
        ka = (((row + 1).astype(np.uint64) << np.uint64(33)) | ((~vec).astype(np.uint64) << np.uint64(32))
              | (prio.astype(np.uint64) << np.uint64(25)) | (off.astype(np.uint64) << np.uint64(1)) | s)
        ka = np.where(seed, np.uint64(2) | s, ka)
        lanes = np.zeros(e.shape, dtype=bool) if lanes is None else np.asarray(lanes, dtype=bool)
        ka = np.where(lanes, np.uint64(0), ka)
    else:
        lanes = np.ones(e.shape, dtype=bool)
    L = rule.lanes
    nv = m - m % L
    vec = off < nv
    lane = np.where(vec, off % L, 0)
    rank = np.where(vec, np.array(rule.rank, dtype=np.int64)[lane], REM_RANK)
    top = ~vec | (rank == 0)
    k1 = np.where(seed | top, ((e + 1).astype(np.uint64) << np.uint64(1)) | s, np.uint64(0))
    inv = (1 << OFF_BITS) - 1 - off
    w = (((row + 1).astype(np.uint64) << np.uint64(32)) | (rank.astype(np.uint64) << np.uint64(25))
         | (inv.astype(np.uint64) << np.uint64(1)) | s)
    w = np.where(seed, s, w)
    k1 = np.where(lanes, k1, np.uint64(0))
    w = np.where(lanes, w, np.uint64(W_NONE))
    return k1, w, ka


def decode_w(w, lr, rule):
    """Reduced position of the element behind a W key."""
    if w < 2:
        return 0
    P = rule.piece
    npr = (lr + P - 1) // P
    row = (int(w) >> 32) - 1
    off = (1 << OFF_BITS) - 1 - ((int(w) >> 1) & ((1 << OFF_BITS) - 1))
    q, k = divmod(row, npr)
    s0 = 1 if (q == 0 and k == 0) else k * P
    return q * lr + s0 + off


def finalize(k1, w, ka, lr, rule):
    """Sign bit from an output's combined keys (None: no zero).  A strided
    call's zero (KA) is always later than the copied first call's."""
    if ka:
        return bool(int(ka) & 1)
    if w == W_NONE and k1 == 0:
        return None
    if k1 == 0:
        return bool(int(w) & 1)
    if w == W_NONE:
        return bool(int(k1) & 1)
    e1 = (int(k1) >> 1) - 1
    return bool(int(w) & 1) if decode_w(w, lr, rule) > e1 else bool(int(k1) & 1)


def predict(arr: np.ndarray, axis, op, rule):
    """Sign of every zero ``op(arr, axis, keepdims=True)`` output by the
    key algorithm, as a dict {output index: sign or None}.  ``arr`` is the
    array NumPy reduces (a view or a copy; its strides decide the walk)."""
    nd = arr.ndim
    red = set(range(nd)) if axis is None else {a % nd for a in (axis if isinstance(axis, tuple) else (axis,))}
    st = [s // arr.itemsize for s in arr.strides]
    perm = sorted(range(nd), key=lambda d: -abs(st[d]))
    mode, lr, n_copy, block = call_structure(arr.shape, st, red, perm, not arr.dtype.isnative, rule.piece)
    rdims = [d for d in perm if d in red]
    kept_red = [d for d in range(nd) if d in red]
    beyond = [d for d in perm if d not in red and d not in block]
    vals = arr if op is np.min else -arr
    out_shape = tuple(1 if d in red else n for d, n in enumerate(arr.shape))
    res = {}
    for o in np.ndindex(out_shape):
        sl = tuple(slice(None) if d in red else o[d] for d in range(nd))
        tr = [kept_red.index(d) for d in rdims]
        sub = np.transpose(np.asarray(vals[sl]), tr).reshape(-1)
        raw = np.transpose(np.asarray(arr[sl]), tr).reshape(-1)
        if np.isnan(sub).any() or sub.min() != 0:
            res[o] = None
            continue
        z = np.flatnonzero(sub == 0)
        lanes = None
        if n_copy and all(o[d] == 0 for d in beyond):
            bidx, f = 0, 1
            for d in block:
                bidx += o[d] * f
                f *= arr.shape[d]
            lanes = (z // lr == 0) & (bidx < n_copy)   # run 0 of a copied output
        k1, w, ka = element_keys(z, np.signbit(raw[z]).astype(np.uint64), mode, lr, rule, lanes)
        res[o] = finalize(k1.max(), w.min(), ka.max(), lr, rule)
    return res


def predict_scan(arr: np.ndarray, axis, op, rule, step: int = 1):
    """:func:`predict` by the device's early-stopping backward scan
    (``k_tie_scan``): each output's reduced positions are visited from the
    last down in steps of ``step``, and the scan stops after the step that
    holds a significant zero of a contiguous call (K1 != 0, not the seed),
    or once the row of the first strided-call zero (KA) is finished; only
    the scanned suffix's keys are finalized.  Returns ``(result, scanned)``:
    the same dict as :func:`predict` and the elements read per output."""
    nd = arr.ndim
    red = set(range(nd)) if axis is None else {a % nd for a in (axis if isinstance(axis, tuple) else (axis,))}
    st = [s // arr.itemsize for s in arr.strides]
    perm = sorted(range(nd), key=lambda d: -abs(st[d]))
    mode, lr, n_copy, block = call_structure(arr.shape, st, red, perm, not arr.dtype.isnative, rule.piece)
    rdims = [d for d in perm if d in red]
    kept_red = [d for d in range(nd) if d in red]
    beyond = [d for d in perm if d not in red and d not in block]
    vals = arr if op is np.min else -arr
    out_shape = tuple(1 if d in red else n for d, n in enumerate(arr.shape))
    res, scanned = {}, {}
    P = rule.piece
    for o in np.ndindex(out_shape):
        sl = tuple(slice(None) if d in red else o[d] for d in range(nd))
        tr = [kept_red.index(d) for d in rdims]
        sub = np.transpose(np.asarray(vals[sl]), tr).reshape(-1)
        raw = np.transpose(np.asarray(arr[sl]), tr).reshape(-1)
        if np.isnan(sub).any() or sub.min() != 0:
            res[o] = None
            continue
        olanes = False
        if n_copy and all(o[d] == 0 for d in beyond):
            bidx, f = 0, 1
            for d in block:
                bidx += o[d] * f
                f *= arr.shape[d]
            olanes = bidx < n_copy
        k1, w, ka = 0, W_NONE, 0
        stop, hi = -1, sub.size
        while hi > 0 and hi > stop:
            lo = max(hi - step, 0)
            e = np.arange(lo, hi, dtype=np.int64)
            zs = e[sub[lo:hi] == 0]
            if zs.size:
                lanes = (olanes & (zs < lr)) if mode == MODE_ACC else None
                x1, xw, xa = element_keys(zs, np.signbit(raw[zs]).astype(np.uint64), mode, lr, rule, lanes)
                k1, w, ka = max(k1, int(x1.max())), min(w, int(xw.min())), max(ka, int(xa.max()))
                acc = (mode == MODE_ACC) & ~(np.zeros(zs.size, bool) if lanes is None else lanes)
                rowst = (zs // lr) * lr + ((zs % lr) // P) * P
                thr = np.where(acc, rowst, np.where((x1 != 0) & (zs > 0), zs, -1))
                stop = max(stop, int(thr.max()))
            hi = lo
        scanned[o] = sub.size - hi
        res[o] = finalize(k1, w, ka, lr, rule)
    return res, scanned


# ---------------------------------------------------------------------------
# host planning of the device passes
# ---------------------------------------------------------------------------
def _sel_tuple(cs):
    out = []
    for d in cs.dims:
        if d.dropped:
            out.append(int(d.start))
        elif d.step == 0:
            out.append(np.asarray(d.indices, dtype=np.intp))
        elif d.count == 0:
            out.append(slice(0, 0))
        else:
            stop = d.start + d.count * d.step
            out.append(slice(d.start, None if stop < 0 else stop, d.step))
    return tuple(out)


def geometry(chunk_shape, order, cs, masked: bool, dtype):
    """``pyas_tie_geom`` of ``chunk[sel]`` after mask_missing
    (storage.py:95-96) in the batch's dim order (dims reversed for an
    F-ordered chunk): the dims from outer to inner in memory, whether NumPy
    reduces the view itself (no mask attribute, slices only: a masked_*
    call or an index list makes a copy, ``np.array(copy=True)`` in 'K'
    order) and whether the byte order forces buffering."""
    from . import _lib
    nd = len(chunk_shape)
    rev = order == "F" and nd > 1
    dev = (lambda k: nd - 1 - k) if rev else (lambda k: k)
    lists = any(d.step == 0 and not d.dropped for d in cs.dims)
    g = _lib.TieGeom()
    if lists:
        # advanced indexing lays the result out by its own rule: ask NumPy
        probe = np.empty(tuple(chunk_shape), dtype=np.uint8, order="F" if rev else "C")[_sel_tuple(cs)]
        st = dict(zip(cs.kept, probe.strides))
        user = [k for k, d in enumerate(cs.dims) if d.dropped] + sorted(cs.kept, key=lambda k: -abs(st[k]))
        perm = [dev(k) for k in user]
    else:
        perm = list(range(nd))
    for i, d in enumerate(perm):
        g.perm[i] = d
    g.flags = (GEOM_VIEW if not masked and not lists else 0) | \
        (GEOM_BUFFERED if not np.dtype(dtype).isnative else 0)
    return g


def grid_lr(extents, reduced) -> int:
    """Reduce-call length over a C-contiguous array of ``extents`` reduced
    over the dims in ``reduced`` (the `out` array of active.py:512,594):
    the product of its trailing reduced extents, 1 when the innermost
    non-1 dim is kept."""
    lr = 1
    for d in range(len(extents) - 1, -1, -1):
        if extents[d] == 1:
            continue
        if d not in reduced:
            break
        lr *= int(extents[d])
    return lr
