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
