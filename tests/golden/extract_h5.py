"""Extract HDF5 chunk tables + raw chunk bytes from the reference's test files.

Runs ONLY in the build container, under ``/opt/conda/bin/python3.9`` (the one
interpreter with h5py 3.3 / libhdf5 1.10.6).  It reads the data files that the
reference's own tests hold (``/root/reference/tests/test_data/*.nc``) and
writes fixtures (data, not code) under ``tests/golden/``:

* ``h5_vars.json``   — per variable: shape, chunk shape, dtype, HDF5 filter
  pipeline, masking attributes, and the chunk index (coords -> offset, size),
  i.e. what pyfive's B-tree walk returns at ``activestorage/active.py:663-665``.
  It also records a SHA-256 of every chunk as decoded by libhdf5 itself, which
  pins the oracle's restated zlib + un-shuffle byte-exactly.
* ``h5_chunks.npz``  — raw (still filtered) chunk bytes, concatenated per variable.
* ``h5_shuffle.npz`` — synthetic datasets written by libhdf5 with the shuffle
  filter (no deflate) for every netCDF numeric type and both byte orders,
  together with the array that was written.

Usage: /opt/conda/bin/python3.9 tests/golden/extract_h5.py
"""
import hashlib
import json
import os
import tempfile

import h5py
import numpy as np

REF = "/root/reference/tests/test_data"
HERE = os.path.dirname(os.path.abspath(__file__))

VARS = [
    ("cesm2_native.nc", "TREFHT"),
    ("daily_data.nc", "ta"),
    ("daily_data_masked.nc", "ta"),
    ("daily_data_fullmask.nc", "ta"),
    ("zero_chunked.nc", "var"),
    ("test1.nc", "tas"),
    ("CMIP6-test.nc", "tas"),
    ("obs4MIPS_CERES-EBAF_L3B_Ed2-8_rlut.nc", "rlut"),
]
# CMIP6_IPSL-CM6A-LR_tas.nc is byte-identical to CMIP6-test.nc (same md5), so
# only the latter is extracted; tests alias the former's known answer to it.
# Raw byte ranges read directly by tests/unit/test_storage.py (file, offset, size).
RAW_RANGES = [
    ("cesm2_native.nc", 2, 128),          # test_storage.py:70-90
    ("daily_data_masked.nc", 6911, 2976),  # test_storage.py:93-119
    ("daily_data_fullmask.nc", 6911, 2976),  # test_storage.py:122-219
    ("zero_chunked.nc", 8760, 48),        # test_storage.py:222-245
]
MASK_ATTRS = ("_FillValue", "missing_value", "valid_min", "valid_max",
              "valid_range")


def attr_json(v):
    a = np.asarray(v)
    return {"dtype": a.dtype.str, "shape": list(a.shape),
            "values": a.reshape(-1).tolist()}


def main():
    meta, blobs = {}, {}
    for fname, vname in VARS:
        path = os.path.join(REF, fname)
        with h5py.File(path, "r") as h, open(path, "rb") as fh:
            ds = h[vname]
            key = f"{fname}:{vname}"
            dcpl = ds.id.get_create_plist()
            filters = []
            for i in range(dcpl.get_nfilters()):
                fid, flags, cd = dcpl.get_filter(i)[:3]
                filters.append({"id": int(fid), "client_data": [int(x) for x in cd]})
            chunks = list(ds.chunks) if ds.chunks else list(ds.shape)
            table, parts, pos = [], [], 0
            if ds.chunks:
                for i in range(ds.id.get_num_chunks()):
                    info = ds.id.get_chunk_info(i)
                    coords = [int(o) // c for o, c in zip(info.chunk_offset, chunks)]
                    fh.seek(info.byte_offset)
                    raw = fh.read(info.size)
                    sl = tuple(slice(o, o + c) for o, c in zip(info.chunk_offset, chunks))
                    dec = np.zeros(chunks, dtype=ds.dtype)
                    got = ds[sl]
                    dec[tuple(slice(0, s) for s in got.shape)] = got
                    table.append({"coords": coords, "offset": int(info.byte_offset),
                                  "size": int(info.size), "filter_mask": int(info.filter_mask),
                                  "blob_start": pos,
                                  "hdf5_decoded_sha256": hashlib.sha256(dec.tobytes()).hexdigest()})
                    parts.append(np.frombuffer(raw, dtype=np.uint8))
                    pos += len(raw)
            else:
                off = ds.id.get_offset()
                size = ds.id.get_storage_size()
                fh.seek(off)
                raw = fh.read(size)
                table.append({"coords": [0] * ds.ndim, "offset": int(off), "size": int(size),
                              "filter_mask": 0, "blob_start": 0,
                              "hdf5_decoded_sha256": hashlib.sha256(ds[...].tobytes()).hexdigest()})
                parts.append(np.frombuffer(raw, dtype=np.uint8))
            attrs = {k: attr_json(ds.attrs[k]) for k in ds.attrs if k in MASK_ATTRS}
            meta[key] = {"file": fname, "var": vname, "shape": list(ds.shape),
                         "chunks": chunks, "chunked": bool(ds.chunks),
                         "dtype": ds.dtype.str, "order": "C", "filters": filters,
                         "attrs": attrs, "chunk_table": table}
            blobs[key] = np.concatenate(parts)
    for fname, off, size in RAW_RANGES:
        with open(os.path.join(REF, fname), "rb") as fh:
            fh.seek(off)
            blobs[f"raw:{fname}:{off}:{size}"] = np.frombuffer(fh.read(size), dtype=np.uint8)
    with open(os.path.join(HERE, "h5_vars.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "h5_chunks.npz"), **blobs)

    # libhdf5-encoded shuffle fixtures: every netCDF numeric type, both orders
    rng = np.random.default_rng(1234)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "shuf.h5")
        with h5py.File(p, "w") as h:
            for code in ("i1", "u1", "i2", "u2", "i4", "u4", "i8", "u8", "f4", "f8"):
                for bo in ("<", ">"):
                    dt = np.dtype(bo + code)
                    if dt.kind == "f":
                        arr = rng.standard_normal((5, 6, 7)).astype(dt) * 100
                    else:
                        info = np.iinfo(dt)
                        arr = rng.integers(info.min, info.max, size=(5, 6, 7),
                                           dtype=np.int64 if dt.kind == "i" else np.uint64,
                                           endpoint=True).astype(dt)
                    name = f"{bo.replace('<', 'le').replace('>', 'be')}_{code}"
                    h.create_dataset(name, data=arr, chunks=(5, 6, 7), shuffle=True,
                                     dtype=dt)
        with h5py.File(p, "r") as h:
            for name in h:
                ds = h[name]
                mask, raw = ds.id.read_direct_chunk((0, 0, 0))
                assert mask == 0
                out[name + ":raw"] = np.frombuffer(raw, dtype=np.uint8)
                out[name + ":data"] = ds[...]
    np.savez_compressed(os.path.join(HERE, "h5_shuffle.npz"), **out)
    print("wrote", len(meta), "variables and", len(out) // 2, "shuffle fixtures")


if __name__ == "__main__":
    main()
