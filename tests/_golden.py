"""Loader for the golden vectors produced by tests/golden/make_golden.py
(outputs of the reference's own storage.py) and tests/golden/extract_h5.py
(libhdf5's own decode of the reference's test files)."""
import functools
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

METHODS = {"ma.sum": np.ma.sum, "ma.min": np.ma.min, "ma.max": np.ma.max, "ma.mean": np.ma.mean,
           "sum": np.sum, "min": np.min, "max": np.max, "mean": np.mean, "none": None}


def dec_value(e):
    if e is None:
        return None
    k = e["kind"]
    if k == "ndarray":
        return np.array(e["v"], dtype=e["dtype"]).reshape(e["shape"])
    if k == "list":
        return list(e["v"])
    if k == "np":
        return np.dtype(e["dtype"]).type(e["v"])
    if k == "int":
        return int(e["v"])
    return float(e["v"])


def dec_sel(e):
    def one(d):
        if "slice" in d:
            return slice(*d["slice"])
        if "ellipsis" in d:
            return Ellipsis
        if "list" in d:
            return list(d["list"])
        return d["int"]
    if "tuple" in e:
        return tuple(one(d) for d in e["tuple"])
    return one(e)


@functools.lru_cache(maxsize=1)
def cases():
    with open(os.path.join(HERE, "reference_cases.json")) as f:
        return json.load(f)["cases"]


@functools.lru_cache(maxsize=1)
def signs_comparable() -> bool:
    """Whether this host's NumPy breaks zero ties as the NumPy that made
    the golden vectors (zerosign.py): then a zero min/max must match its
    sign bit too (the device follows the host's rule)."""
    from pyactivestorage_amd.zerosign import tie_rule
    with open(os.path.join(HERE, "reference_cases.json")) as f:
        rec = json.load(f).get("tie_rule", {})
    for dt in ("f4", "f8"):
        r = tie_rule(dt)
        if r is None or dt not in rec or rec[dt] != {"lanes": r.lanes, "order": r.order, "piece": r.piece,
                                                     "acc": r.acc, "acc_order": r.acc_order}:
            return False
    return True


@functools.lru_cache(maxsize=1)
def arrays():
    return dict(np.load(os.path.join(HERE, "reference_outputs.npz")))


@functools.lru_cache(maxsize=1)
def h5_meta():
    with open(os.path.join(HERE, "h5_vars.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=1)
def h5_blobs():
    return dict(np.load(os.path.join(HERE, "h5_chunks.npz")))


def args_of(i, zlib_cls, shuffle_cls):
    """Replay arguments of golden case i for a reduce_chunk_bytes-like call."""
    c = cases()[i]
    raw = arrays()[c["input"]].tobytes()
    comp = zlib_cls() if c["codecs"].get("zlib") else None
    filters = [shuffle_cls(c["codecs"]["shuffle"])] if c["codecs"].get("shuffle") else None
    missing = tuple(dec_value(v) for v in c["missing"])
    axis = tuple(c["axis"]) if c["axis"] is not None else None
    return dict(raw=raw, compression=comp, filters=filters, missing=missing, dtype=c["dtype"],
                shape=tuple(c["shape"]), order=c["order"], chunk_selection=dec_sel(c["sel"]),
                axis=axis, method=METHODS[c["method"]])


def expected(i):
    """(expect-dict, data, mask, count) of golden case i (or raises name)."""
    c = cases()[i]
    if "raises" in c:
        return c["raises"], None, None, None
    a = arrays()
    return c["expect"], a[f"data{i}"], a[f"mask{i}"], a.get(f"count{i}")


SUM_METHODS = ("ma.sum", "sum", "ma.mean", "mean")


def check(i, tmp, n, rel=1e-6):
    """Assert (tmp, n) reproduces golden case i.  Containers, dtypes, shapes,
    masks and counts exactly; float sums/means within ``rel`` (0: exact);
    every other value (min/max, integer results) byte for byte, NaN as NaN,
    and a zero min/max down to its sign bit wherever this host breaks zero
    ties as the generating host did (storage.py:99-100)."""
    exp, data, mask, count = expected(i)
    assert type(tmp).__name__ == exp["type"], (i, type(tmp), exp)
    assert np.asarray(tmp).dtype.str == exp["dtype"] or np.dtype(exp["dtype"]) == tmp.dtype, (i, tmp.dtype, exp)
    assert list(np.shape(tmp)) == exp["shape"], (i, np.shape(tmp), exp)
    if exp["type"] == "MaskedArray":
        assert (np.ma.getmask(tmp) is np.ma.nomask) == exp["nomask"], (i, "nomask", exp)
    gm = np.ma.getmaskarray(tmp)
    assert np.array_equal(gm, mask), (i, gm, mask)
    gd = np.asarray(np.ma.getdata(tmp))[~mask]
    wd = data[~mask]
    if wd.dtype.kind == "f" and rel and cases()[i]["method"] in SUM_METHODS:
        w, g = wd.astype(np.float64), gd.astype(np.float64)
        ok = (np.isnan(w) & np.isnan(g)) | (w == g) | (np.abs(w - g) <= rel * np.abs(w))
        assert ok.all(), (i, gd, wd)
    elif wd.dtype.kind == "f":
        gn, wn = np.isnan(gd), np.isnan(wd)
        assert np.array_equal(gn, wn), (i, "nan", gd, wd)
        g8, w8 = gd[~gn].astype(wd.dtype), wd[~wn]
        z = w8 == 0
        if not signs_comparable():   # compare zeros by value only
            assert np.array_equal(g8[z], w8[z]), (i, gd, wd)
            g8, w8 = g8[~z], w8[~z]
        assert g8.tobytes() == w8.tobytes(), (i, "bytes", gd, wd)
    else:
        assert gd.astype(wd.dtype).tobytes() == wd.tobytes(), (i, gd, wd)
    if count is None:
        assert n is None, i
    else:
        assert n.dtype == count.dtype and np.array_equal(n, count), (i, n, count)


def check_gpu(i, tmp, n, a, reduce_bytes):
    """:func:`check` at 1e-6 relative; float sums/means that cancel may
    instead sit within 4e-7 * sum|x| of the reference (NumPy's pairwise f32
    error bound, tests/_compare.py) -- only where the sum really cancels
    (|sum| < sum|x| / 2): a non-cancelling sum is held to 1e-6.  Returns
    True when case i needed that fallback (the caller reports how many did)."""
    try:
        check(i, tmp, n, rel=1e-6)
        return False
    except AssertionError:
        c = cases()[i]
        if c["method"] not in SUM_METHODS:
            raise
    sel, _ = reduce_bytes(a["raw"], a["compression"], a["filters"], a["missing"], a["dtype"],
                          a["shape"], a["order"], a["chunk_selection"], None, None)
    with np.errstate(all="ignore"):
        scale = np.ma.sum(np.abs(np.ma.asarray(sel).astype(np.float64)), axis=a["axis"], keepdims=True)
    _, data, mask, count = expected(i)
    g = np.asarray(np.ma.getdata(tmp), dtype=np.float64)[~mask]
    w = data.astype(np.float64)[~mask]
    s = np.broadcast_to(np.ma.filled(scale, 0), mask.shape)[~mask]
    with np.errstate(invalid="ignore"):
        strict = (np.isnan(g) & np.isnan(w)) | (np.abs(g - w) <= 1e-6 * np.abs(w))
        ok = strict | ((np.abs(g - w) <= 4e-7 * s) & (np.abs(w) < 0.5 * s))
    assert ok.all(), (i, g, w)
    assert np.array_equal(np.ma.getmaskarray(tmp), mask) and np.array_equal(n, count), i
    return True
