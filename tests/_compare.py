"""Parity assertions between the HIP path and the oracle (test helper)."""
import numpy as np


def shuffle_bytes(arr: np.ndarray, es: int) -> bytes:
    """HDF5/numcodecs shuffle *encode* (inverse of the decode under test)."""
    raw = np.frombuffer(arr.tobytes(), dtype=np.uint8)
    n = raw.size // es
    return raw[: n * es].reshape(n, es).T.reshape(-1).tobytes() + raw[n * es:].tobytes()


# Float sums/means: NumPy sums float32 pairwise in float32, the GPU in float64
# and rounds once; both are within a few ulp of the exact value, so we allow
# 1e-6 relative (north_star's bound) or, where the sum cancels, 4e-7 of the
# sum of |x| (NumPy pairwise error bound for these sizes).
REL_TOL = 1e-6
ABS_FRAC = 4e-7


def assert_same(want, got, kind=None, data_abs_sum=None, what=""):
    """Reference result vs GPU result: same container, dtype, shape, mask;
    values bit-exact except float sums/means."""
    assert type(got) is type(want), f"{what}: type {type(got)} != {type(want)}"
    assert got.dtype == want.dtype, f"{what}: dtype {got.dtype} != {want.dtype}"
    assert got.shape == want.shape, f"{what}: shape {got.shape} != {want.shape}"
    keep = np.ones(want.shape, dtype=bool)
    if isinstance(want, np.ma.MaskedArray):
        wm, gm = np.ma.getmask(want), np.ma.getmask(got)
        assert (wm is np.ma.nomask) == (gm is np.ma.nomask), f"{what}: nomask mismatch {wm!r} {gm!r}"
        wma, gma = np.ma.getmaskarray(want), np.ma.getmaskarray(got)
        assert np.array_equal(wma, gma), f"{what}: mask {gma} != {wma}"
        keep = ~wma
    wd = np.asarray(np.ma.getdata(want))[keep]
    gd = np.asarray(np.ma.getdata(got))[keep]
    if wd.dtype.kind == "f" and kind in ("sum", "mean", None):
        w64, g64 = wd.astype(np.float64), gd.astype(np.float64)
        tol = REL_TOL * np.abs(w64)
        if data_abs_sum is not None:
            s = np.broadcast_to(np.asarray(data_abs_sum, dtype=np.float64), want.shape)[keep]
            tol = np.maximum(tol, ABS_FRAC * s)
        with np.errstate(invalid="ignore"):
            ok = (np.isnan(g64) & np.isnan(w64)) | (g64 == w64) | (np.abs(g64 - w64) <= tol)
        assert ok.all(), f"{what}: values {gd[~ok]} != {wd[~ok]} (tol {tol[~ok]})"
    else:
        assert np.array_equal(gd, wd, equal_nan=wd.dtype.kind == "f"), f"{what}: {gd} != {wd}"


def assert_counts(want_n, got_n, what=""):
    if want_n is None:
        assert got_n is None, what
        return
    assert type(got_n) is type(want_n), f"{what}: count type {type(got_n)} != {type(want_n)}"
    assert got_n.dtype == want_n.dtype and got_n.shape == want_n.shape, what
    assert np.array_equal(got_n, want_n), f"{what}: counts {got_n} != {want_n}"


def oracle_partials(arr, sel, axis, missing):
    """Per-output (count, sum, min, max) of one chunk straight from the
    oracle (``oracle.storage_ref.reduce_chunk_bytes``: ``chunk[sel]``, then
    mask_missing, storage.py:95-100), C order over the kept dims.  Sums in
    the class accumulator (f64 / i64 / u64); min/max in the native dtype,
    NaN where an unmasked NaN is present.  For checking a kernel's raw
    per-output partials against the reference semantics directly."""
    from oracle import storage_ref as ref
    dt = arr.dtype
    nd = dt.newbyteorder("=")
    if missing is None:
        missing = (None, None, None, None)
    vals, _ = ref.reduce_chunk_bytes(arr.tobytes(), None, None, missing, dt.str, arr.shape, "C", sel, axis, None)
    m = np.ma.getmaskarray(vals)
    vm = np.ma.MaskedArray(np.ma.getdata(vals).astype(nd), mask=m)
    acc = np.float64 if dt.kind == "f" else (np.int64 if dt.kind == "i" else np.uint64)
    out = {"count": (~m).sum(axis=axis, keepdims=True).reshape(-1)}
    out["sum"] = np.ma.filled(vm.astype(acc), 0).sum(axis=axis, keepdims=True).reshape(-1)
    with np.errstate(invalid="ignore"):
        out["min"] = np.ma.getdata(np.ma.min(vm, axis=axis, keepdims=True)).reshape(-1)
        out["max"] = np.ma.getdata(np.ma.max(vm, axis=axis, keepdims=True)).reshape(-1)
    return out


def assert_partials_match_oracle(parts, want, dt, what, rtol=1e-6):
    """Kernel partials (engine.partial_dtype rows) vs oracle_partials: count
    exact, min/max equal where count > 0 (NaN where NumPy gives NaN; the
    sign of a zero extreme is fixed later by the zero-sign passes, so values
    compare equal here), sums within rtol (floats) or exact."""
    nd = dt.newbyteorder("=")
    np.testing.assert_array_equal(parts["count"], want["count"], err_msg=f"{what}: count")
    ok = want["count"] > 0
    for k in ("min", "max"):
        g = parts[k][ok].astype(nd)
        w = want[k][ok]
        if dt.kind == "f":
            np.testing.assert_array_equal(np.isnan(g), np.isnan(w), err_msg=f"{what}: {k} NaN")
            fin = ~np.isnan(w)
            np.testing.assert_array_equal(g[fin], w[fin], err_msg=f"{what}: {k}")
        else:
            np.testing.assert_array_equal(g, w, err_msg=f"{what}: {k}")
    if dt.kind == "f":
        g, w = parts["sum"][ok].astype(np.float64), want["sum"][ok]
        fin = np.isfinite(w)
        np.testing.assert_allclose(g[fin], w[fin], rtol=rtol, atol=1e-3, err_msg=f"{what}: sum")
    else:
        np.testing.assert_array_equal(parts["sum"][ok], want["sum"][ok], err_msg=f"{what}: sum")
