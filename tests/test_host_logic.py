"""CPU-only tests of the host logic around the kernels: the mask compiler
(exact NumPy-promotion thresholds), selection normalisation, result
formatting, and the C-ABI library surface (loads, exports every symbol
declared in include/pyas.h, reports errors without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import _lib, results, selection
from pyactivestorage_amd.masking import compile_missing

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DTYPES = ["<f4", ">f4", "<f8", "<i2", ">i2", "<u2", "<i4", "<u4", "<i8", "<u8", "i1", "u1"]


def _device_mask(cm, x):
    """What the kernel computes (pyas_device.hpp MaskT::masked), in NumPy on
    the storage dtype, from the compiled thresholds."""
    nd = cm.dt.newbyteorder("=")
    x = x.astype(nd)
    m = np.zeros(x.shape, dtype=bool)
    with np.errstate(invalid="ignore"):
        for k, bit in ((0, _lib.MASK_EQ0), (1, _lib.MASK_EQ1)):
            if cm.flags & bit:
                lo, hi = cm.eq[k]
                m |= (x >= nd.type(lo)) & (x <= nd.type(hi))
        if cm.flags & _lib.MASK_GT:
            m |= x > nd.type(cm.gt)
        if cm.flags & _lib.MASK_LT:
            m |= x < nd.type(cm.lt)
    return m


def _probe_values(dt, value):
    """Values of dt around `value` and around the type limits."""
    dt = np.dtype(dt)
    nd = dt.newbyteorder("=")
    out = []
    if nd.kind == "f":
        for v in (value, 0.0, -0.0, np.inf, -np.inf, np.nan, 1e20, -999.0, 0.1, 5e8, 1000.0):
            try:
                c = nd.type(v)
            except (OverflowError, ValueError):
                continue
            out.append(c)
            a = c
            b = c
            for _ in range(3):
                a = np.nextafter(a, nd.type(np.inf))
                b = np.nextafter(b, nd.type(-np.inf))
                out += [a, b]
    else:
        info = np.iinfo(nd)
        cands = [info.min, info.min + 1, info.max, info.max - 1, 0, 1, -1, 42, 25, 1000, -999]
        try:
            v = int(np.floor(float(value)))
            cands += [v - 2, v - 1, v, v + 1, v + 2]
        except (OverflowError, ValueError, TypeError):
            pass
        out = [c for c in cands if info.min <= c <= info.max]
    return np.array(out, dtype=nd).astype(dt)


VALUES = [42, 42.0, 42.5, -7, 0.1, 1e20, np.float32(0.1), np.float64(1e20), np.float32(1e20), np.int16(42),
          np.uint8(200), 2 ** 40, -1e30, 1e30, np.inf, -np.inf, np.nan, 0.0, -0.0, np.float64(-999.0)]


@pytest.mark.parametrize("dt", DTYPES)
def test_mask_compiler_matches_numpy(dt):
    """For each rule, the device test on the compiled threshold selects exactly
    the elements NumPy's masked_equal/greater/less select (storage.py:126-153)."""
    for v in VALUES:
        for slot in range(4):
            missing = [None, None, None, None]
            missing[slot] = v
            try:
                want_fn = ref.mask_missing
                x = _probe_values(dt, v)
                want = np.ma.getmaskarray(want_fn(x.copy(), tuple(missing)))
            except Exception as exc:  # the compiler must raise the same way
                with pytest.raises(type(exc)):
                    compile_missing(tuple(missing), dt)
                continue
            cm = compile_missing(tuple(missing), dt)
            got = _device_mask(cm, x)
            assert np.array_equal(got, want), (dt, slot, v, x[got != want])


def test_mask_compiler_vectors():
    cm = compile_missing((None, [42.0, 43.0, 1e20], None, None), "<f4")
    assert cm.flags & _lib.MASK_TAB1
    lo, hi, ok = cm.tables[1]
    assert list(ok) == [True, True, False]
    cm = compile_missing(([7], None, None, None), "<i2")  # 1-element list -> scalar slot
    assert cm.flags & _lib.MASK_EQ0 and cm.eq[0] == (7, 7)


def _apply(cs, arr):
    """Host emulation of the device's per-dim (start, step, count) selection."""
    idx = []
    for d in cs.dims:
        if d.step == 0:
            idx.append(np.asarray(d.indices))
        else:
            idx.append(d.start + d.step * np.arange(d.count))
    sub = arr[np.ix_(*idx)]
    return sub.reshape(cs.shape)


SELS = [
    (slice(None),) * 3, (slice(1, 4), slice(None), slice(0, 7, 2)), (2, slice(None), slice(1, 5)),
    (slice(None), [0, 2, 3], slice(None)), (slice(4, 0, -1), slice(None), slice(None)),
    slice(0, 2, 1), (Ellipsis, 3), (Ellipsis,), (-1, -2, slice(None, None, -3)), (slice(7, 2),),
    (np.array([4, 0]), slice(None), slice(None)), (slice(None), np.array([True, False, True, True]), 0),
    (np.int64(2), slice(1, 3), slice(None)),
]


@pytest.mark.parametrize("k", range(len(SELS)))
def test_selection_normalize_matches_numpy(k):
    arr = np.arange(5 * 4 * 7).reshape(5, 4, 7)
    cs = selection.normalize(SELS[k], arr.shape)
    want = arr[SELS[k]]
    assert cs.shape == want.shape
    assert np.array_equal(_apply(cs, arr), want)


def test_selection_errors_match_numpy():
    arr = np.zeros((3, 4))
    for bad in ((3, 0), (0, slice(None), 1), ([0, 5], slice(None))):
        with pytest.raises(IndexError):
            arr[bad]
        with pytest.raises(IndexError):
            selection.normalize(bad, arr.shape)


def test_selection_pack_layout():
    cs = [selection.normalize((slice(1, 3), [0, 2], 1), (4, 3, 2)),
          selection.normalize((slice(None), slice(None), slice(None)), (4, 3, 2))]
    table, pool = selection.pack(cs, 3)
    assert table.shape == (2, _lib.MAX_DIMS, 3) and table.dtype == np.int32
    assert list(table[0, 0]) == [1, 1, 2] and list(table[0, 1]) == [0, 0, 2] and list(table[0, 2]) == [1, 1, 1]
    assert list(pool[:2]) == [0, 2]
    assert list(table[1, 2]) == [0, 1, 2] and list(table[0, 5]) == [0, 1, 1]


@pytest.mark.parametrize("dt", ["<f4", ">f8", "<i2", "<u1", "<i8"])
@pytest.mark.parametrize("method", [np.ma.sum, np.ma.min, np.ma.max, np.ma.mean, np.sum, np.mean, np.max])
@pytest.mark.parametrize("missing", [(None, None, None, None), (3, None, None, None),
                                     (1e20, None, None, None), (None, None, 2, 9)])
def test_results_formatting_matches_numpy(dt, method, missing):
    """results.build on exact partials gives the reference's container, dtype,
    shape, mask (incl. nomask shrink) and values (storage.py:98-100)."""
    rng = np.random.default_rng(1)
    arr = rng.integers(0, 12, size=(3, 4, 5)).astype(dt)
    for axis in (None, (1,), (0, 2)):
        try:
            want, wn = ref.reduce_chunk_bytes(arr.tobytes(), None, None, missing, dt, arr.shape, "C",
                                              (slice(None),) * 3, axis, method)
        except TypeError:  # e.g. fill 1e20 on int16: the mask compiler test covers raising
            return
        masked = ref.mask_missing(arr.copy(), missing)
        ax = axis if axis is not None else (0, 1, 2)
        keep = tuple(1 if i in ax else n for i, n in enumerate(arr.shape))
        nd = np.dtype(dt).newbyteorder("=")
        from pyactivestorage_amd.engine import partial_dtype
        parts = np.zeros(keep, dtype=partial_dtype(dt))
        data = np.ma.asarray(masked).astype(nd)
        cnt = np.ma.count(data, axis=ax, keepdims=True)
        parts["count"] = cnt
        s = np.ma.sum(data.astype(np.float64 if nd.kind == "f" else (np.int64 if nd.kind == "i" else np.uint64)),
                      axis=ax, keepdims=True)
        parts["sum"] = np.ma.filled(s, 0)
        if cnt.min() > 0:
            parts["min"] = np.ma.min(data, axis=ax, keepdims=True)
            parts["max"] = np.ma.max(data, axis=ax, keepdims=True)
        kind, is_ma = results.method_kind(method)
        n_red = int(np.prod([arr.shape[i] for i in ax]))
        got, gn = results.build(parts, kind, is_ma, dt, any(m is not None for m in missing), n_red, arr.size)
        assert type(got) is type(want) and got.dtype == want.dtype and got.shape == want.shape
        if isinstance(want, np.ma.MaskedArray):
            assert (np.ma.getmask(got) is np.ma.nomask) == (np.ma.getmask(want) is np.ma.nomask)
            assert np.array_equal(np.ma.getmaskarray(got), np.ma.getmaskarray(want))
        w = np.ma.filled(want.astype(np.float64), 0) if want.dtype.kind == "f" else np.ma.filled(want, 0)
        g = np.ma.filled(got.astype(np.float64), 0) if got.dtype.kind == "f" else np.ma.filled(got, 0)
        np.testing.assert_allclose(g, w, rtol=1e-6)
        assert np.array_equal(gn, wn)


def test_method_kind():
    assert results.method_kind(np.ma.sum) == ("sum", True)
    assert results.method_kind(np.amin) == ("min", False)
    assert results.method_kind("mean") == ("mean", True)
    with pytest.raises(NotImplementedError):
        results.method_kind(np.median)
    with pytest.raises(ValueError):
        results.method_kind("median")


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "pyas.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(pyas_\w+)\s*\(", text, re.M)))


def test_capi_exports_every_declared_symbol():
    lib = _lib.load()
    syms = _declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, s  # and the ctypes binding covers it
    assert set(_lib.SIGNATURES) == set(syms)


def test_capi_struct_layouts():
    assert ctypes.sizeof(_lib.Partial) == 32
    assert ctypes.sizeof(_lib.Scalar) == 8
    assert _lib.Batch.data.offset == 4 * 4 + 8 * _lib.MAX_DIMS + 8
    assert ctypes.sizeof(_lib.Mask) == 4 + 8 + 16 + 16 + 8 + 8 + 16 + 16 + 2 * 8 * _lib.MAX_DIMS + 4  # padding
    assert ctypes.sizeof(_lib.TieGeom) == 4 * _lib.MAX_DIMS + 4
    assert ctypes.sizeof(_lib.TieRule) == 3 * 4 + 64 + 64
    assert ctypes.sizeof(_lib.ChunkDesc) == 4 * 4 + 8 * _lib.MAX_DIMS + 4 + 4 + 4 + ctypes.sizeof(_lib.TieGeom)
    from pyactivestorage_amd import _fastpath   # the C side's own sizeof
    assert _fastpath.CHUNK_DESC_SIZE == ctypes.sizeof(_lib.ChunkDesc)


def test_capi_errors_without_gpu_are_reported():
    lib = _lib.load()
    assert lib.pyas_abi_version() == _lib.ABI_VERSION
    n = ctypes.c_int(-1)
    rc = lib.pyas_device_count(ctypes.byref(n))
    if rc != _lib.OK:  # no GPU in the build container: error + message, no crash
        assert n.value == 0 and lib.pyas_last_error()
    assert lib.pyas_device_count(None) == _lib.EINVAL
    assert b"NULL" in lib.pyas_last_error()
    # NULL context -> EINVAL on every entry point that takes one
    assert lib.pyas_reduce_chunks(None, None, None, None, None, 0, None) == _lib.EINVAL
    assert lib.pyas_combine_partials(None, 0, None, 0, 0, None, None) == _lib.EINVAL
    with pytest.raises(ValueError):
        _lib.check(_lib.EINVAL)
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.ENOTSUP)


def test_inflate_status_mapping_and_packing():
    """pyas_inflate statuses map to zlib.decompress's exceptions (storage.py:119-120)."""
    import zlib as _z

    from pyactivestorage_amd.inflate import pack_streams, raise_for_status
    cap = np.array([8, 8, 8], dtype=np.int64)
    raise_for_status(np.zeros(3, np.int32), cap, cap)   # all OK: no exception
    for code, text in ((1, "incorrect header check"), (8, "incomplete or truncated stream"),
                       (9, "incorrect data check"), (7, "invalid distance too far back")):
        with pytest.raises(_z.error, match=text):
            raise_for_status(np.array([0, code, 0], np.int32), cap, cap)
    with pytest.raises(_z.error, match="^Error 2 while decompressing data$"):
        raise_for_status(np.array([2], np.int32), cap[:1], cap[:1])
    with pytest.raises(ValueError):
        raise_for_status(np.array([10], np.int32), cap[:1], cap[:1])
    host, offs, sizes = pack_streams([b"abc", b"", b"defgh"], align=4)
    assert list(offs) == [0, 4, 4] and list(sizes) == [3, 0, 5]
    assert host[:3].tobytes() == b"abc" and host[4:9].tobytes() == b"defgh"


def _state(x):
    if isinstance(x, np.ma.MaskedArray):
        d = dict(x.__dict__)
        m = d.pop("_mask")
        return (type(x), x.dtype.str, x.shape, np.asarray(x.data).tobytes(), m is np.ma.nomask,
                np.asarray(m).tobytes(), sorted(d.items(), key=lambda kv: kv[0]).__repr__())
    return (type(x), x.dtype.str, x.shape, np.asarray(x).tobytes())


@pytest.mark.parametrize("dt", ["<f4", ">f8", "<i2", "<u4", "<i8", "u1"])
def test_build_one_matches_build(dt):
    """The drop-in's single-partial result builder returns objects identical
    to the generic one (type, dtype, shape, data, mask, MaskedArray state)."""
    from pyactivestorage_amd.engine import partial_dtype
    pdt = partial_dtype(dt)
    p = np.zeros(1, dtype=pdt)
    cls = pdt["sum"].type
    for cnt, n_sel in ((5, 5), (3, 5), (0, 5)):
        p["count"] = cnt
        p["sum"] = cls(1234) if np.dtype(dt).kind != "f" else 1234.5678901234
        p["min"] = cls(7)
        p["max"] = cls(99)
        for shape in ((1,), (1, 1, 1)):
            for kind in ("sum", "min", "max", "mean"):
                for is_ma in (True, False):
                    for rule in (True, False):
                        if not rule and cnt < n_sel:
                            continue
                        want = results.build(p.reshape(shape), kind, is_ma, np.dtype(dt), rule, n_sel, n_sel)
                        got = results.build_one(p[0], shape, kind, is_ma, np.dtype(dt), rule, n_sel, n_sel)
                        assert _state(got[0]) == _state(want[0]), (dt, cnt, kind, is_ma, rule)
                        assert _state(got[1]) == _state(want[1])


def test_inflate_choice(monkeypatch):
    """Active's device/host inflate choice (row f3): forced
    either way, or by stream count against the measured crossover per host
    lane (active.py inflate_on_device), PYAS_ACTIVE_INFLATE overriding auto."""
    from pyactivestorage_amd import active as A
    monkeypatch.delenv("PYAS_ACTIVE_INFLATE", raising=False)
    assert A.inflate_on_device(1, 30, True) and not A.inflate_on_device(10_000, 30, False)
    n_cross = int(A._INFLATE_CROSSOVER * min(30, A._INGEST_LANES))
    assert not A.inflate_on_device(n_cross - 1, 30, "auto")
    assert A.inflate_on_device(n_cross, 30, "auto")
    assert not A.inflate_on_device(n_cross - 1, 4, "auto") or n_cross - 1 >= A._INFLATE_CROSSOVER * 4
    monkeypatch.setenv("PYAS_ACTIVE_INFLATE", "device")
    assert A.inflate_on_device(1, 30, "auto")
    monkeypatch.setenv("PYAS_ACTIVE_INFLATE", "host")
    assert not A.inflate_on_device(10_000, 30, "auto") and A.inflate_on_device(1, 30, True)
    nc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nc", "test1.nc")
    with pytest.raises(ValueError):
        A.Active(nc, "tas", device_inflate="gpu")


def _sel_table(rows):
    t = np.zeros((len(rows), 8, 3), dtype=np.int32)
    for i, r in enumerate(rows):
        for d in range(8):
            t[i, d] = r[d] if d < len(r) else (0, 1, 1)
    return t


@pytest.mark.parametrize("rows,dense,none", [
    ([[(0, 1, 4), (0, 1, 8), (0, 1, 16)]], True, False),            # whole chunk
    ([[(1, 1, 3), (0, 1, 8), (0, 1, 16)]], True, False),            # a box over half of it
    ([[(0, 1, 4), (0, 1, 8), (3, 1, 1)]], False, True),             # a thin box: generic walk
    ([[(0, 1, 4), (0, 3, 3), (0, 1, 16)]], False, True),            # strided kept dim
    ([[(0, 1, 4), (0, 0, 2), (0, 1, 16)]], False, True),            # an index list
    ([[(0, 1, 4), (0, 3, 3), (0, 1, 16)], [(0, 1, 4), (0, 1, 8), (0, 1, 16)]], False, False),   # mixed
    ([[(0, 1, 4), (0, 1, 8), (0, 1, 1)]], False, True),             # one innermost index: under half
])
def test_dense_classes(rows, dense, none):
    """ReductionPlan's promises to pyas_reduce_axes_ex (PYAS_REC_DENSE_ONLY /
    PYAS_REC_GENERIC_ONLY): they must mirror the kernels' chunk ownership
    (pyas_kernels.hpp chunk_is_full / cut_eligible), or outputs go unwritten."""
    from pyactivestorage_amd.batch import ReductionPlan

    class P:
        chunk_shape = (4, 8, 16)
    p = P()
    p.sel_table_host = _sel_table(rows)
    ReductionPlan._dense_class(p)
    assert p._dense_boxes == dense and p._no_dense == none
