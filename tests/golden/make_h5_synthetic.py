"""Synthetic HDF5 files for the metadata reader (pyactivestorage_amd/hdf5.py),
written by libhdf5 itself, with the answers libhdf5 gives for them.

Runs ONLY in the build container under /opt/conda/bin/python3.9 (h5py 3.3,
libhdf5 1.10.6).  Writes tests/golden/h5synth/*.h5 and h5synth.json:
per dataset its shape, chunk shape, dtype, filter pipeline, numeric
attributes and chunk table (h5py's get_chunk_info), covering what the
reference's own files do not: superblock v0 with a symbol-table group of
many datasets, big-endian and integer types, dense attributes, nested
groups, dense links, compact and contiguous layouts, and a libver-latest
file (layout v4) the reader must refuse by name.

Usage: /opt/conda/bin/python3.9 tests/golden/make_h5_synthetic.py
"""
import json
import os

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "h5synth")


def describe(path, name):
    with h5py.File(path, "r") as f:
        d = f[name]
        pl = d.id.get_create_plist()
        filters = []
        for i in range(pl.get_nfilters()):
            fid, _flags, vals, _name = pl.get_filter(i)
            filters.append({"id": int(fid), "client_data": [int(v) for v in vals]})
        table = []
        if d.chunks is not None:
            for i in range(d.id.get_num_chunks()):
                ci = d.id.get_chunk_info(i)
                table.append({"coords": [o // c for o, c in zip(ci.chunk_offset, d.chunks)],
                              "offset": int(ci.byte_offset), "size": int(ci.size)})
        else:
            off = d.id.get_offset()
            table.append({"coords": [0] * d.ndim, "offset": None if off is None else int(off),
                          "size": int(d.id.get_storage_size())})
        attrs = {}
        for k, v in d.attrs.items():
            a = np.asarray(v)
            if a.dtype.kind in "iuf":
                attrs[k] = {"dtype": a.dtype.str, "shape": list(a.shape), "values": a.reshape(-1).tolist()}
        return {"file": os.path.basename(path), "var": name, "shape": list(d.shape),
                "chunks": list(d.chunks) if d.chunks else list(d.shape), "dtype": d.dtype.str,
                "layout": int(pl.get_layout()), "filters": filters, "attrs": attrs, "chunk_table": table}


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(0)
    cases = []

    p = os.path.join(OUT, "v0_symtab.h5")                    # superblock v0, old-style groups
    with h5py.File(p, "w", libver="earliest") as f:
        for i in range(12):
            f.create_dataset(f"d{i:02d}", data=rng.normal(size=(4, 6)).astype("<f4"), chunks=(2, 3))
        d = f.create_dataset("tas", data=rng.normal(size=(10, 20, 30)).astype("<f4"), chunks=(5, 10, 15),
                             compression="gzip", compression_opts=3, shuffle=True)
        d.attrs["_FillValue"] = np.float32(1e20)
        d.attrs["valid_range"] = np.array([-5, 5], dtype="<f4")
        for i in range(6):
            d.attrs[f"note{i}"] = f"text {i}"
    cases += [(p, "tas"), (p, "d07")]

    p = os.path.join(OUT, "v108_dense.h5")                   # superblock v2, dense attrs, nested group
    with h5py.File(p, "w", libver=("v108", "v110")) as f:
        g = f.create_group("g1").create_group("g2")
        d = g.create_dataset("ts", data=rng.integers(-300, 300, size=(50, 40)).astype(">i2"),
                             chunks=(16, 16), compression="gzip", compression_opts=1)
        for i in range(12):
            d.attrs[f"a{i}"] = np.int32(i)
        d.attrs["missing_value"] = np.int16(-999)
        d.attrs["valid_min"] = np.int16(-250)
        c = f.create_dataset("compact", data=np.arange(10, dtype="<f8"),
                             **({} if not hasattr(h5py.h5d, "COMPACT") else {}))
        f.create_dataset("contig", data=rng.normal(size=(7, 9)).astype(">f8"))
        for i in range(30):                                     # dense links in the root group
            f.create_dataset(f"x{i:02d}", data=np.arange(i + 1, dtype="<u8"), chunks=(1,))
    cases += [(p, "g1/g2/ts"), (p, "contig"), (p, "x17"), (p, "compact")]

    p = os.path.join(OUT, "v108_compact.h5")                 # compact layout
    with h5py.File(p, "w", libver=("v108", "v110")) as f:
        sp = h5py.h5s.create_simple((6, 4))
        pl = h5py.h5p.create(h5py.h5p.DATASET_CREATE)
        pl.set_layout(h5py.h5d.COMPACT)
        dsid = h5py.h5d.create(f.id, b"small", h5py.h5t.NATIVE_INT32, sp, pl)
        dsid.write(h5py.h5s.ALL, h5py.h5s.ALL, np.arange(24, dtype="<i4").reshape(6, 4))
    cases += [(p, "small")]

    p = os.path.join(OUT, "v108_big_btrees.h5")               # v2 B-trees with internal nodes
    with h5py.File(p, "w", libver=("v108", "v110")) as f:
        for i in range(400):                                    # dense links, depth >= 1 name index
            f.create_dataset(f"var{i:03d}", data=np.full((3,), i, dtype="<i4"), chunks=(3,))
        d = f.create_dataset("many_attrs", data=np.arange(12, dtype="<f4").reshape(3, 4), chunks=(3, 2))
        for i in range(3000):                                   # dense attributes, depth 2 name index
            d.attrs[f"attr{i:04d}"] = np.float64(i) / 7
        d.attrs["_FillValue"] = np.float32(-1.0)
    cases += [(p, "var000"), (p, "var257"), (p, "var399"), (p, "many_attrs")]

    p = os.path.join(OUT, "latest.h5")                        # layout v4 chunk indexes
    with h5py.File(p, "w", libver="latest") as f:
        f.create_dataset("v", data=np.zeros((8, 8), "<f4"), chunks=(4, 4), maxshape=(None, 8))  # extensible array
        f.create_dataset("fa", data=rng.normal(size=(20, 30)).astype("<f4"), chunks=(8, 8))       # fixed array
        f.create_dataset("fa_z", data=rng.normal(size=(20, 30)).astype(">f8"), chunks=(8, 8),
                         compression="gzip", shuffle=True)                                         # filtered
        f.create_dataset("fa_paged", data=np.arange(2500 * 4, dtype="<i2").reshape(2500, 4),
                         chunks=(1, 4))                                                            # > 1024 entries
        f.create_dataset("single", data=rng.normal(size=(6, 7)).astype("<f4"), chunks=(6, 7))
        f.create_dataset("single_z", data=rng.normal(size=(6, 7)).astype("<f4"), chunks=(6, 7),
                         compression="gzip")
        dcpl = h5py.h5p.create(h5py.h5p.DATASET_CREATE)
        dcpl.set_chunk((4, 5))
        dcpl.set_alloc_time(h5py.h5d.ALLOC_TIME_EARLY)
        sid = h5py.h5s.create_simple((12, 10))
        dsid = h5py.h5d.create(f.id, b"implicit", h5py.h5t.IEEE_F32LE, sid, dcpl=dcpl)
        dsid.write(h5py.h5s.ALL, h5py.h5s.ALL, rng.normal(size=(12, 10)).astype("<f4"))
        # extensible arrays: one unlimited dim, first or not; enough chunks to
        # fill the index block, index-block data blocks, super blocks, pages
        f.create_dataset("ea", data=rng.normal(size=(10, 8)).astype("<f4"), chunks=(3, 4),
                         maxshape=(None, 8))
        f.create_dataset("ea_big", data=np.arange(6000 * 3, dtype="<i4").reshape(6000, 3), chunks=(1, 3),
                         maxshape=(None, 3))
        f.create_dataset("ea_z", data=rng.normal(size=(300, 6)).astype("<f8"), chunks=(2, 3),
                         maxshape=(None, 6), compression="gzip")
        # unlimited dim not first: libhdf5 1.10.6's H5Dget_chunk_info reports
        # these chunks' offsets swizzled, so the test checks chunk contents
        # (arange data) instead of that table
        f.create_dataset("ea_mid", data=np.arange(4 * 50 * 5, dtype="<f4").reshape(4, 50, 5),
                         chunks=(2, 1, 5), maxshape=(4, None, 5))
    cases += [(p, n) for n in ("fa", "fa_z", "fa_paged", "single", "single_z", "implicit",
                               "v", "ea", "ea_big", "ea_z", "ea_mid")]
    p = os.path.join(OUT, "latest_2unlim.h5")                 # v2 B-tree chunk index
    with h5py.File(p, "w", libver="latest") as f:
        f.create_dataset("v", data=rng.normal(size=(8, 8)).astype("<f4"), chunks=(4, 4),
                         maxshape=(None, None))
        f.create_dataset("many", data=np.arange(60 * 70, dtype="<i2").reshape(60, 70), chunks=(2, 3),
                         maxshape=(None, None))                                  # internal nodes
        f.create_dataset("many_z", data=rng.normal(size=(40, 50)).astype("<f8"), chunks=(3, 4),
                         maxshape=(None, None), compression="gzip", shuffle=True)  # filtered records
    cases += [(p, n) for n in ("v", "many", "many_z")]
    out = {f"{os.path.basename(a)}:{b}": describe(a, b) for a, b in cases}
    with open(os.path.join(HERE, "h5synth.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", len(out), "datasets")


if __name__ == "__main__":
    main()
