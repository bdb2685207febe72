"""GPU parity of the drop-in ``reduce_chunk`` against the oracle.

Template: the reference's exhaustive sweep ``tests/unit/test_active_axis.py:30-78``
(index patterns x axis permutations x methods, exact mask and count equality)
applied at the ``storage.reduce_chunk`` level (``storage.py:8-104``) across all
ten netCDF numeric dtypes, both byte orders, with and without the shuffle
filter, and every masking attribute.
"""
import itertools
import zlib

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import storage as pas
from tests._compare import assert_counts, assert_same, shuffle_bytes

pytestmark = pytest.mark.gpu

DTYPES = ["<f4", ">f4", "<f8", ">f8", "<i2", ">i2", "<u2", "<i4", ">u4", "<i8", "<u8", "i1", "u1"]
SHAPE = (6, 5, 7)

SELECTIONS = [
    (slice(0, 6, 1), slice(0, 5, 1), slice(0, 7, 1)),      # full chunk
    (slice(1, 4, 1), slice(0, 5, 1), slice(0, 7, 1)),      # contiguous rows
    (slice(0, 6, 2), slice(1, 5, 3), slice(0, 7, 4)),      # strided
    (slice(2, 3, 1), slice(0, 5, 1), slice(2, 6, 1)),      # one row, inner run
    (slice(5, 0, -2), slice(None), slice(6, None, -1)),    # negative steps
    (3, slice(0, 5, 1), slice(1, 7, 1)),                   # integer drops axis 0
    (slice(None), [0, 1, 4], slice(None)),                 # list index
    slice(0, 2, 1),                                        # bare slice (test_storage.py:85)
    (Ellipsis, slice(2, 5)),
]


def _data(dt, rng, nan=False):
    dt = np.dtype(dt)
    if dt.kind == "f":
        a = rng.uniform(-50, 150, size=SHAPE).astype(dt)
        a.reshape(-1)[::11] = 42.0
        if nan:
            a.reshape(-1)[7] = np.nan
    else:
        info = np.iinfo(dt)
        lo, hi = max(info.min, -300), min(info.max, 300)
        a = rng.integers(lo, hi, size=SHAPE, endpoint=True).astype(dt)
        a.reshape(-1)[::11] = 42
    return a


def _missings(dt):
    dt = np.dtype(dt)
    base = [
        (None, None, None, None),
        (42, None, None, None),                                  # python int fill
        (None, np.array([42], dtype=dt), None, None),            # 1-element vector
        (42.0, None, 0, 100),                                    # fill + valid range
        (None, 42, None, 120),
        (-7, None, 10, None),
    ]
    if dt.kind == "f":
        base += [
            (0.1, None, None, 0.1),                               # f64 promotion
            (np.float32(42.0), None, np.float64(-1e30), np.float64(1e30)),
            (None, [42.0, 43.0, 44.0, 45.0, 46.0, 47.0, 48.0], None, None),  # broadcast vector
            (1e20, 1e20, None, None),                             # non-representable in f32
        ]
    else:
        base += [
            (None, None, None, -1e30),                            # everything masked
            (None, [42, 43, 44, 45, 46, 47, 48], None, None),
        ]
    return base


AXES_FOR = {3: [None, (0, 1, 2), (1,), (0, 2), (2, 0), (-1,)], 2: [None, (0, 1), (0,), (1,)]}
METHODS = [np.ma.sum, np.ma.min, np.ma.max, np.ma.mean, np.sum, np.mean, np.max]


def _cases():
    rng = np.random.default_rng(7)
    out = []
    for dt in DTYPES:
        for shuf in (False, True):
            for k, sel in enumerate(SELECTIONS):
                for miss in _missings(dt):
                    out.append((dt, shuf, k, miss))
    # deterministic thinning to keep the run short
    rng.shuffle(out)
    return out[:900]


CASES = _cases()


def _run_pair(raw, filters, miss, dt, sel, axis, method):
    want, wn = ref.reduce_chunk_bytes(raw, None, filters and [ref.Shuffle(f.elementsize) for f in filters],
                                      miss, dt, SHAPE, "C", sel, axis, method)
    got, gn = pas.reduce_chunk_bytes(raw, None, filters, miss, dt, SHAPE, "C", sel, axis, method)
    return want, wn, got, gn


@pytest.mark.parametrize("case", range(len(CASES)))
def test_reduce_chunk_matches_oracle(gpu, case):
    dt, shuf, k, miss = CASES[case]
    sel = SELECTIONS[k]
    rng = np.random.default_rng(case)
    arr = _data(dt, rng, nan=(case % 5 == 0))
    es = np.dtype(dt).itemsize
    raw = shuffle_bytes(arr, es) if shuf else arr.tobytes()
    filters = [pas.Shuffle(es)] if shuf else None
    sub_ndim = len(ref.decode_chunk(arr.tobytes(), None, None, dt, SHAPE, "C")[sel].shape)
    for axis in AXES_FOR.get(sub_ndim, [None]):
        for method in METHODS:
            what = f"{dt} shuf={shuf} sel={sel} miss={miss} axis={axis} {method.__name__}"
            try:
                want, wn, got, gn = _run_pair(raw, filters, miss, dt, sel, axis, method)
            except (ValueError, IndexError, TypeError) as exc:  # both sides must raise alike
                with pytest.raises(type(exc)):
                    pas.reduce_chunk_bytes(raw, None, filters, miss, dt, SHAPE, "C", sel, axis, method)
                continue
            masked_sel, _ = ref.reduce_chunk_bytes(raw, None, filters and [ref.Shuffle(es)], miss, dt,
                                                   SHAPE, "C", sel, axis, None)
            with np.errstate(all="ignore"):
                abs_sum = np.ma.sum(np.abs(np.ma.asarray(masked_sel).astype(np.float64)),
                                    axis=axis, keepdims=True)
            kind = method.__name__.replace("amin", "min").replace("amax", "max")
            assert_same(want, got, kind, np.ma.filled(abs_sum, 0), what)
            assert_counts(wn, gn, what)


@pytest.mark.parametrize("dt", DTYPES)
def test_select_method_none(gpu, dt):
    """method=None returns the masked selection itself (storage.py:95-103)."""
    rng = np.random.default_rng(3)
    arr = _data(dt, rng)
    for shuf in (False, True):
        es = np.dtype(dt).itemsize
        raw = shuffle_bytes(arr, es) if shuf else arr.tobytes()
        filters = [pas.Shuffle(es)] if shuf else None
        for sel in SELECTIONS:
            for miss in _missings(dt)[:4]:
                want, wn = ref.reduce_chunk_bytes(raw, None, filters and [ref.Shuffle(es)], miss, dt,
                                                  SHAPE, "C", sel, None, None)
                got, gn = pas.reduce_chunk_bytes(raw, None, filters, miss, dt, SHAPE, "C", sel, None, None)
                assert gn is None and wn is None
                assert type(got) is type(want) and got.dtype == want.dtype and got.shape == want.shape
                if isinstance(want, np.ma.MaskedArray):
                    assert np.array_equal(np.ma.getmaskarray(got), np.ma.getmaskarray(want))
                assert np.array_equal(np.asarray(got), np.asarray(want), equal_nan=arr.dtype.kind == "f")


def test_fortran_order(gpu):
    rng = np.random.default_rng(11)
    arr = rng.uniform(0, 10, size=SHAPE).astype("<f4")
    raw = np.asfortranarray(arr).tobytes(order="A")
    for sel in SELECTIONS[:5]:
        for axis in (None, (1,), (0, 2)):
            for method in (np.ma.sum, np.ma.max):
                want, wn = ref.reduce_chunk_bytes(raw, None, None, (None, None, 2.0, None), "<f4", SHAPE,
                                                  "F", sel, axis, method)
                got, gn = pas.reduce_chunk_bytes(raw, None, None, (None, None, 2.0, None), "<f4", SHAPE,
                                                 "F", sel, axis, method)
                assert_same(want, got, "sum", None, f"F {sel} {axis}")
                assert_counts(wn, gn)


def test_file_reduce_chunk_roundtrip(gpu, tmp_path):
    """The file-reading entry point: read_block + reduce (storage.py:51-62)."""
    rng = np.random.default_rng(5)
    arr = rng.uniform(0, 10, size=(4, 8, 8)).astype("<f8")
    path = tmp_path / "chunks.bin"
    pad = b"\x00" * 13
    path.write_bytes(pad + arr.tobytes())
    sel = (slice(0, 4, 1), slice(1, 7, 1), slice(0, 8, 2))
    want, wn = ref.reduce_chunk(str(path), 13, arr.nbytes, None, None, (None, None, None, 9.0), "<f8",
                                (4, 8, 8), "C", sel, (0, 1, 2), np.ma.max)
    got, gn = pas.reduce_chunk(str(path), 13, arr.nbytes, None, None, (None, None, None, 9.0), "<f8",
                               (4, 8, 8), "C", sel, (0, 1, 2), np.ma.max)
    assert_same(want, got, "max")
    assert_counts(wn, gn)


def test_file_reduce_chunk_pinned_staging(gpu, tmp_path):
    """reduce_chunk's file read goes into a per-thread pinned staging buffer
    (storage.py:51-53 read_block): growing chunk sizes from one thread, a
    zlib + shuffle chunk (device inflate straight from the staging view),
    eight threads at once on different chunks, and a read past the end of
    the file (storage.py:57-62 raises ValueError on the short reshape)."""
    import concurrent.futures
    from oracle.storage_ref import Shuffle, Zlib
    rng = np.random.default_rng(9)
    shapes = [(2, 4, 4), (16, 32, 32), (8, 8, 8), (64, 64, 64), (4, 4, 4)]
    arrs = [rng.uniform(-5, 5, size=s).astype("<f4") for s in shapes]
    comp = zlib.compress(shuffle_bytes(arrs[1], 4), 4)
    blobs = [a.tobytes() for a in arrs] + [comp]
    offs, pos = [], 7
    path = tmp_path / "mixed.bin"
    with open(path, "wb") as fh:
        fh.write(b"\x01" * 7)
        for b in blobs:
            offs.append(pos)
            fh.write(b)
            pos += len(b)
    miss = (None, None, -4.0, 4.0)
    sel_of = lambda s: tuple(slice(0, n, 1) for n in s)

    def one(k):
        s = shapes[k]
        want, wn = ref.reduce_chunk(str(path), offs[k], len(blobs[k]), None, None, miss, "<f4", s, "C",
                                    sel_of(s), (0, 1, 2), np.ma.sum)
        got, gn = pas.reduce_chunk(str(path), offs[k], len(blobs[k]), None, None, miss, "<f4", s, "C",
                                   sel_of(s), (0, 1, 2), np.ma.sum)
        assert_same(want, got, "sum")
        assert_counts(wn, gn, f"chunk {k}")

    for k in range(len(shapes)):            # one thread, staging grows and is reused
        one(k)
    zc, filt = Zlib(4), [Shuffle(4)]
    want, wn = ref.reduce_chunk(str(path), offs[-1], len(comp), zc, filt, miss, "<f4", shapes[1], "C",
                                sel_of(shapes[1]), (0, 1, 2), np.ma.max)
    got, gn = pas.reduce_chunk(str(path), offs[-1], len(comp), zc, filt, miss, "<f4", shapes[1], "C",
                               sel_of(shapes[1]), (0, 1, 2), np.ma.max)
    assert_same(want, got, "max")
    assert_counts(wn, gn, "zlib+shuffle")
    with concurrent.futures.ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(one, [k % len(shapes) for k in range(40)]))
    for fn in (ref.reduce_chunk, pas.reduce_chunk):   # past the end of the file
        with pytest.raises(ValueError):
            fn(str(path), pos - 100, len(blobs[0]) + 200, None, None, miss, "<f4", (2, 4, 4), "C",
               sel_of((2, 4, 4)), (0, 1, 2), np.ma.sum)
