"""Generate golden vectors by running the REFERENCE's own storage.reduce_chunk.

Runs only in the build container (needs /root/reference).  The reference's
``activestorage/storage.py`` is loaded by file path with two import stubs
(``pyfive`` is only used in a ``type(rfile) is ...`` check at storage.py:46,
and ``numcodecs.compat.ensure_ndarray`` becomes ``np.frombuffer``); codecs
passed in are the oracle's restatements of numcodecs Zlib/Shuffle (pinned
against libhdf5 by ``extract_h5.py``).  Nothing from the reference is copied:
the outputs are data (inputs + expected outputs) in ``reference_outputs.npz``
and ``reference_cases.json``.

Usage: python tests/golden/make_golden.py
"""
import contextlib
import hashlib
import importlib.util
import io
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_STORAGE = "/root/reference/activestorage/storage.py"
sys.path.insert(0, ROOT)

from oracle import storage_ref  # noqa: E402  (codec restatements only)


def load_reference_storage():
    pyfive = types.ModuleType("pyfive")
    hl = types.ModuleType("pyfive.high_level")

    class Dataset:  # storage.py:46 type check only
        pass
    hl.Dataset = Dataset
    pyfive.high_level = hl
    numcodecs = types.ModuleType("numcodecs")
    compat = types.ModuleType("numcodecs.compat")
    compat.ensure_ndarray = lambda b: b if isinstance(b, np.ndarray) else np.frombuffer(memoryview(b), "u1")
    numcodecs.compat = compat
    sys.modules.update({"pyfive": pyfive, "pyfive.high_level": hl, "numcodecs": numcodecs,
                        "numcodecs.compat": compat})
    spec = importlib.util.spec_from_file_location("reference_storage", REF_STORAGE)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# ---------------------------------------------------------------------------
# JSON encodings that replay with exact Python/NumPy types
# ---------------------------------------------------------------------------
def enc_value(v):
    if v is None:
        return None
    if isinstance(v, np.ndarray):
        return {"kind": "ndarray", "dtype": v.dtype.str, "shape": list(v.shape), "v": v.reshape(-1).tolist()}
    if isinstance(v, list):
        return {"kind": "list", "v": v}
    if isinstance(v, np.generic):
        return {"kind": "np", "dtype": np.dtype(type(v)).str, "v": v.item()}
    if isinstance(v, bool):
        raise TypeError
    if isinstance(v, int):
        return {"kind": "int", "v": v}
    if isinstance(v, float):
        return {"kind": "float", "v": repr(v)}
    raise TypeError(type(v))


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


def enc_sel(sel):
    def one(s):
        if isinstance(s, slice):
            return {"slice": [s.start, s.stop, s.step]}
        if s is Ellipsis:
            return {"ellipsis": True}
        if isinstance(s, (list, np.ndarray)):
            return {"list": [int(x) for x in np.asarray(s).reshape(-1)]}
        return {"int": int(s)}
    if isinstance(sel, tuple):
        return {"tuple": [one(s) for s in sel]}
    return one(sel)


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


METHODS = {"ma.sum": np.ma.sum, "ma.min": np.ma.min, "ma.max": np.ma.max, "ma.mean": np.ma.mean,
           "sum": np.sum, "min": np.min, "max": np.max, "mean": np.mean, "none": None}


def codecs(spec):
    comp = storage_ref.Zlib() if spec.get("zlib") else None
    filters = [storage_ref.Shuffle(spec["shuffle"])] if spec.get("shuffle") else None
    return comp, filters


def run_case(ref, raw, case):
    """The reference's own ``reduce_chunk`` (storage.py:8-104) on `raw`
    written to a temporary file, called as active.py:765-776 calls it."""
    comp, filters = codecs(case["codecs"])
    missing = tuple(dec_value(v) for v in case["missing"])
    axis = tuple(case["axis"]) if case["axis"] is not None else None
    fd, path = tempfile.mkstemp(suffix=".chunk")
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(raw)
        with contextlib.redirect_stdout(io.StringIO()):  # storage.py:44 prints per chunk
            return ref.reduce_chunk(path, 0, len(raw), comp, filters, missing, np.dtype(case["dtype"]),
                                    tuple(case["shape"]), case["order"], dec_sel(case["sel"]), axis,
                                    method=METHODS[case["method"]])
    finally:
        os.unlink(path)


def describe(out):
    tmp, n = out
    d = {"type": type(tmp).__name__, "dtype": np.asarray(tmp).dtype.str if not isinstance(tmp, np.ma.MaskedArray)
         else tmp.dtype.str, "shape": list(np.shape(tmp))}
    if isinstance(tmp, np.ma.MaskedArray):
        m = np.ma.getmask(tmp)
        d["nomask"] = m is np.ma.nomask
    return d


def main():
    ref = load_reference_storage()
    rng = np.random.default_rng(2024)
    cases, arrays = [], {}

    def add(raw, **kw):
        idx = len(cases)
        case = dict(kw)
        case["missing"] = [enc_value(v) for v in kw["missing"]]
        case["sel"] = enc_sel(kw["sel"])
        case.setdefault("codecs", {})
        key = "in_" + hashlib.sha1(raw).hexdigest()[:16]   # inputs shared by several cases
        arrays.setdefault(key, np.frombuffer(raw, dtype=np.uint8))
        case["input"] = key
        try:
            tmp, n = run_case(ref, raw, case)
        except Exception as exc:  # the reference's own error is the expected output
            case["raises"] = type(exc).__name__
            cases.append(case)
            return
        case["expect"] = describe((tmp, n))
        arrays[f"data{idx}"] = np.ascontiguousarray(np.ma.getdata(tmp))
        arrays[f"mask{idx}"] = np.ascontiguousarray(np.ma.getmaskarray(tmp))
        if n is not None:
            arrays[f"count{idx}"] = np.ascontiguousarray(n)
        cases.append(case)

    # 1. the reference's own unit-test inputs (tests/unit/test_storage.py)
    blobs = np.load(os.path.join(HERE, "h5_chunks.npz"))
    cesm = blobs["raw:cesm2_native.nc:2:128"].tobytes()
    add(cesm, source="tests/unit/test_storage.py:70-90", dtype="i2", shape=[8, 8], order="C",
        sel=slice(0, 2, 1), axis=[0, 1], method="min", missing=[None, 2050, None, None])
    dm = blobs["raw:daily_data_masked.nc:6911:2976"].tobytes()
    full4 = (slice(0, 62, 1), slice(0, 2, 1), slice(0, 3, 1), slice(0, 2, 1))
    add(dm, source="tests/unit/test_storage.py:93-119", dtype="float32", shape=[62, 2, 3, 2], order="C",
        sel=full4, axis=[0, 1, 2, 3], method="mean", missing=[None, 999.0, None, None])
    fm = blobs["raw:daily_data_fullmask.nc:6911:2976"].tobytes()
    for src, miss in (("122-144", [None, 999.0, None, None]), ("147-169", [999.0, None, None, None]),
                      ("172-194", [None, None, 1000.0, None]), ("197-219", [None, None, None, 1.0])):
        add(fm, source=f"tests/unit/test_storage.py:{src}", dtype="float32", shape=[62, 2, 3, 2],
            order="C", sel=full4, axis=[0, 1, 2, 3], method="mean", missing=miss)
    zc = blobs["raw:zero_chunked.nc:8760:48"].tobytes()
    add(zc, source="tests/unit/test_storage.py:222-245", dtype="float32", shape=[3, 4], order="C",
        sel=(slice(0, 3, 1), slice(0, 4, 1)), axis=[0, 1], method="mean", missing=[None, None, None, None])
    # test_mask_missing broadcast semantics (test_storage.py:9-67) as reductions
    d = np.array([[[-900., 33.], [33., -900], [33., 44.]]], dtype="<f8")
    for miss in ([[-900.], np.array([-900.]), None, None], [[-900., 33.], np.array([-900., 33.]), None, None],
                 [-900, np.array([-900., 33.]), None, None], [-900, np.array([-900., -900., 33.]), None, None]):
        for meth in ("ma.sum", "none"):
            add(d.tobytes(), source="tests/unit/test_storage.py:9-67", dtype="<f8", shape=[1, 3, 2],
                order="C", sel=(slice(None),) * 3, axis=[0, 1, 2], method=meth, missing=miss)

    # 2. real files: every test1.nc chunk (zlib + shuffle, f8) and cesm2 chunks
    meta = json.load(open(os.path.join(HERE, "h5_vars.json")))
    t1 = meta["test1.nc:tas"]
    blob = blobs["test1.nc:tas"]
    for ch in t1["chunk_table"]:
        raw = blob[ch["blob_start"]: ch["blob_start"] + ch["size"]].tobytes()
        for meth, axis in (("ma.min", [0, 1, 2]), ("ma.max", [0, 1, 2]), ("ma.sum", [0, 2]), ("ma.mean", [1])):
            add(raw, source="tests/test_data/test1.nc:tas (tests/unit/test_active_axis.py:94-116)",
                dtype="<f8", shape=t1["chunks"], order="C", sel=(slice(None),) * 3, axis=axis, method=meth,
                codecs={"zlib": True, "shuffle": 8},
                missing=[np.float64(1.00000002e+20), np.float64(1.00000002e+20), None, None])
    ce = meta["cesm2_native.nc:TREFHT"]
    blob = blobs["cesm2_native.nc:TREFHT"]
    for ch in ce["chunk_table"][:6]:
        raw = blob[ch["blob_start"]: ch["blob_start"] + ch["size"]].tobytes()
        add(raw, source="tests/test_data/cesm2_native.nc:TREFHT (tests/test_bigger_data.py:261-284)",
            dtype="<f4", shape=ce["chunks"], order="C", sel=(slice(0, 1), slice(1, 2), slice(None)),
            axis=[0, 1, 2], method="ma.sum", missing=[np.float32(-900.0), np.float32(-900.0), None, None])

    # 3. synthetic sweep: dtypes x byte order x shuffle x masks x selections x methods
    dtypes = ["<f4", ">f4", "<f8", ">f8", "<i2", ">i2", "<u2", "<i4", ">u4", "<i8", "<u8", "i1", "u1"]
    sels = [(slice(None),) * 3, (slice(1, 4), slice(None), slice(0, 7, 2)), (2, slice(None), slice(1, 5)),
            (slice(None), [0, 2, 3], slice(None)), (slice(4, 0, -1), slice(None), slice(None))]
    for dt in dtypes:
        ndt = np.dtype(dt)
        if ndt.kind == "f":
            arr = rng.uniform(-100, 300, size=(5, 4, 7)).astype(ndt)
            arr.reshape(-1)[::9] = 25.0
            arr.reshape(-1)[5] = np.nan
            misses = [[None, None, None, None], [25.0, None, 0.0, 200.0], [np.float32(25.0), 0.1, None, None],
                      [None, [25.0, 26.0, 27.0, 28.0, 29.0, 30.0, 31.0], None, None]]
        else:
            info = np.iinfo(ndt)
            arr = rng.integers(max(info.min, -200), min(info.max, 200), size=(5, 4, 7), endpoint=True).astype(ndt)
            arr.reshape(-1)[::9] = 25
            misses = [[None, None, None, None], [25, None, 0, 150], [None, 25.5, None, -1e30],
                      [None, [25, 26, 27, 28, 29, 30, 31], None, None]]
        for shuffle in (False, True):
            es = ndt.itemsize
            raw = arr.tobytes()
            if shuffle and es > 1:
                b = np.frombuffer(raw, dtype=np.uint8)
                raw = b.reshape(-1, es).T.reshape(-1).tobytes()
            for miss in misses:
                for sel in sels:
                    for meth, axis in (("ma.sum", None), ("ma.min", [0, 2]), ("ma.max", [1]),
                                       ("ma.mean", None), ("mean", [0]), ("max", None)):
                        add(raw, source="synthetic", dtype=dt, shape=[5, 4, 7], order="C", sel=sel,
                            axis=axis, method=meth, missing=miss,
                            codecs={"shuffle": es} if shuffle and es > 1 else {})

    # 4. zero extremes with both signed zeros (storage.py:99-100 np.ma.min/max
    #    and np.min/max): NumPy's sign of a zero min/max follows its reduction
    #    loop (pyactivestorage_amd/zerosign.py).  Data >= 0 (min is a zero),
    #    <= 0 (max is a zero), and all zeros; > np.getbufsize() elements so
    #    the iterator's piece boundary is crossed; masked (the filled copy
    #    NumPy reduces is contiguous) and unmasked whole-chunk selections.
    zshape = (6, 10, 160)
    for dt in ("<f4", ">f4", "<f8", ">f8"):
        ndt = np.dtype(dt)
        for pattern in ("min0", "max0", "zeros"):
            n = int(np.prod(zshape))
            if pattern == "zeros":
                arr = np.zeros(n, dtype=ndt)
            else:
                arr = rng.uniform(0.5, 400.0, n).astype(ndt) * (1 if pattern == "min0" else -1)
            pos = rng.choice(n, 40, replace=False)
            arr[pos] = np.where(rng.random(40) < 0.5, -0.0, 0.0)
            arr[rng.choice(n, 30, replace=False)] = -999.0
            arr[0] = -0.0 if pattern != "max0" else 0.0
            arr = arr.reshape(zshape)
            for shuffle in ((False, True) if dt == "<f4" else (False,)):
                es = ndt.itemsize
                raw = arr.tobytes()
                if shuffle:
                    raw = np.frombuffer(raw, dtype=np.uint8).reshape(-1, es).T.reshape(-1).tobytes()
                for miss in ([None, None, None, None], [-999.0, None, None, None], [None, -999.0, -1.0, 1e6],
                             [-999.0, None, -500.0, 500.0]):
                    sels = [(slice(None),) * 3]
                    if miss[0] is not None or miss[1] is not None:
                        sels.append((slice(1, 6), slice(2, 9), slice(3, 150, 2)))   # masked: filled copy
                    for sel in sels:
                        for meth in ("ma.min", "ma.max", "min", "max"):
                            add(raw, source="zero-sign", dtype=dt, shape=list(zshape), order="C", sel=sel,
                                axis=[0, 1, 2], method=meth, missing=miss,
                                codecs={"shuffle": es} if shuffle else {})

    # 5. signed zeros over axis subsets and strided / listed selections: per
    #    output NumPy visits the reduced elements in its iterator's order
    #    (elementwise when the innermost dim is kept, reduce calls over the
    #    trailing reduced dims otherwise), and an unmasked selection is
    #    reduced as the strided view itself (zerosign.py).  Dense signed
    #    zeros so most outputs are a zero.
    axsets = [[0], [1], [2], [0, 1], [1, 2], [0, 2], [0, 1, 2]]
    zsels = [(slice(None),) * 3, (slice(1, 7), slice(0, 11, 2), slice(3, 37)),
             (slice(7, 0, -2), slice(None), slice(38, 2, -3)), (slice(None), [0, 3, 4, 9], slice(5, 30)),
             (slice(2, 5), slice(None), slice(None, None, 4))]
    zshape2 = (8, 12, 40)
    for dt in ("<f4", "<f8", ">f8", "<f4s"):
        shuffle = dt.endswith("s")
        ndt = np.dtype(dt.rstrip("s"))
        for pattern in ("min0", "max0", "zeros"):
            n = int(np.prod(zshape2))
            arr = np.zeros(n, dtype=ndt) if pattern == "zeros" else \
                rng.uniform(0.5, 400.0, n).astype(ndt) * (1 if pattern == "min0" else -1)
            z = rng.random(n) < 0.3
            arr[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
            arr[rng.choice(n, 25, replace=False)] = -999.0
            arr = arr.reshape(zshape2)
            raw = arr.tobytes()
            es = ndt.itemsize
            if shuffle:
                raw = np.frombuffer(raw, dtype=np.uint8).reshape(-1, es).T.reshape(-1).tobytes()
            for miss in ([None, None, None, None], [-999.0, None, -500.0, 500.0]):
                for sel in zsels:
                    for axis in axsets:
                        for meth in (("ma.min", "max") if pattern != "max0" else ("ma.max", "min")):
                            add(raw, source="zero-sign-axes", dtype=dt.rstrip("s"), shape=list(zshape2), order="C",
                                sel=sel, axis=axis, method=meth, missing=miss,
                                codecs={"shuffle": es} if shuffle else {})
    # reduce calls longer than np.getbufsize() (pieces inside a call)
    zshape3 = (3, 40, 300)
    for dt in ("<f4", ">f8"):
        ndt = np.dtype(dt)
        for pattern in ("min0", "zeros"):
            n = int(np.prod(zshape3))
            arr = np.zeros(n, dtype=ndt) if pattern == "zeros" else rng.uniform(0.5, 400.0, n).astype(ndt)
            k = 60 if pattern == "min0" else n // 3
            pos = rng.choice(n, k, replace=False)
            arr[pos] = np.where(rng.random(k) < 0.5, -0.0, 0.0)
            if pattern == "zeros":
                arr[:] = np.where(rng.random(n) < 0.5, -0.0, 0.0)
            raw = arr.reshape(zshape3).tobytes()
            for miss in ([None, None, None, None], [-999.0, None, None, None]):
                for sel in ((slice(None),) * 3, (slice(None), slice(0, 40, 3), slice(None))):
                    for axis in ([1, 2], [2], [0, 2], [0, 1, 2]):
                        for meth in ("ma.min", "min"):
                            add(raw, source="zero-sign-axes", dtype=dt, shape=list(zshape3), order="C", sel=sel,
                                axis=axis, method=meth, missing=miss)

    sys.path.insert(0, ROOT)
    from pyactivestorage_amd.zerosign import tie_rule
    rules = {dt: {"lanes": r.lanes, "order": r.order, "piece": r.piece, "acc": r.acc, "acc_order": r.acc_order}
             for dt, r in (("f4", tie_rule("f4")), ("f8", tie_rule("f8"))) if r is not None}
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "reference": REF_STORAGE,
                   "numpy": np.__version__, "tie_rule": rules, "cases": cases}, f)
    np.savez_compressed(os.path.join(HERE, "reference_outputs.npz"), **arrays)
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
