"""One Active query shape over the C3 variable attached resident (as
bench.py's c3_slab / c3_stride extras), repeated: for rocprofv3 kernel
splits of a single query shape.

    python tools/query_c3.py NAME LABEL_INDEX [--reps 10]
    e.g. python tools/query_c3.py c3_slab 4     (the 5th query of c3_slab)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("which", type=int)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--zeros", type=float, default=0.0,
                    help="fraction of elements set to +-0.0 (random signs; a zero-heavy field)")
    ap.add_argument("--method", default=None, help="override the query's method (e.g. min)")
    ap.add_argument("--tile-bytes", type=int, default=0, help="pyas_ctx_set_tile_bytes (0: the default)")
    a = ap.parse_args()
    import torch
    from pyactivestorage_amd.active import Active, attach_resident, release_resident
    from pyactivestorage_amd.synthetic import chunk_major_device
    from pyactivestorage_amd.variable import ChunkedVariable
    cfg = bench.CONFIGS["c3"]
    dt = np.dtype(cfg["dtype"])
    shape, chunks = cfg["shape"], cfg["chunks"]
    dev = torch.device("cuda", 0)
    data, offsets, _ = chunk_major_device(torch, shape, chunks, dt, dev, fill=bench.FILL, fill_frac=0.01, seed=0)
    if a.zeros > 0:   # values in [1, 1000) with a fraction of +-0.0, on the device
        v = data.view(torch.float32)
        g = torch.Generator(device="cuda")
        g.manual_seed(1)
        step = 1 << 26
        for i in range(0, v.numel(), step):
            part = v[i:i + step]
            u = torch.rand(part.numel(), generator=g, device="cuda")
            sg = torch.rand(part.numel(), generator=g, device="cuda") < 0.5
            vals = 1.0 + torch.rand(part.numel(), generator=g, device="cuda") * 999.0
            z = torch.where(sg, torch.tensor(-0.0, device="cuda"), torch.tensor(0.0, device="cuda"))
            part.copy_(torch.where(u < a.zeros, z, vals))
    torch.cuda.synchronize()
    grid = [s // c for s, c in zip(shape, chunks)]
    cb = int(np.prod(chunks)) * dt.itemsize
    index = {co: (int(offsets[k]), cb) for k, co in enumerate(np.ndindex(*grid))}
    attrs = {"_FillValue": np.array([bench.FILL], dtype=dt), "valid_min": np.array([bench.VMIN], dtype=dt),
             "valid_max": np.array([bench.VMAX], dtype=dt)}
    if a.zeros > 0:   # the zero-heavy field: _FillValue only (bench_zeros.py's variable)
        attrs = {"_FillValue": np.array([bench.FILL], dtype=dt)}
    var = ChunkedVariable(name="q", shape=shape, chunks=chunks, dtype=dt, chunk_index=index, attrs=attrs,
                          filename=None, filter_pipeline=None)
    attach_resident(var, data.data_ptr(), device=0, owner=data)
    if a.tile_bytes:
        from pyactivestorage_amd.device import get_context
        get_context(0).set_tile_bytes(a.tile_bytes)
    label, mk, axis, method = bench.ACTIVE_EXTRAS[a.name][a.which]
    method = a.method or method
    ix = mk()
    act = Active(var, resident=True)
    times = []
    for _ in range(a.reps + 2):
        getattr(act, method)(axis=axis)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        act[ix]
        times.append(time.perf_counter() - t0)
    times = times[2:]
    print(json.dumps({"query": label, "axis": axis, "method": method, "zeros": a.zeros,
                      "ms_median": round(float(np.median(times)) * 1e3, 4),
                      "ms_min": round(min(times) * 1e3, 4)}), flush=True)
    release_resident(var)


if __name__ == "__main__":
    main()
