"""cProfile of one bench.py Active extra query (C3 attached resident): where
an end-to-end query's host time goes."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    from pyactivestorage_amd.active import Active, attach_resident, release_resident
    from pyactivestorage_amd.synthetic import chunk_major_device
    from pyactivestorage_amd.variable import ChunkedVariable
    cfg = bench.CONFIGS["c3"]
    dt = np.dtype(cfg["dtype"])
    shape, chunks = cfg["shape"], cfg["chunks"]
    dev = torch.device("cuda", 0)
    data, offsets, _ = chunk_major_device(torch, shape, chunks, dt, dev, fill=bench.FILL, fill_frac=0.01, seed=0)
    grid = [s // c for s, c in zip(shape, chunks)]
    cb = int(np.prod(chunks)) * dt.itemsize
    index = {co: (int(offsets[k]), cb) for k, co in enumerate(np.ndindex(*grid))}
    attrs = {"_FillValue": np.array([bench.FILL], dtype=dt)}
    var = ChunkedVariable(name="p", shape=shape, chunks=chunks, dtype=dt, chunk_index=index, attrs=attrs,
                          filename=None, filter_pipeline=None)
    attach_resident(var, data.data_ptr(), device=0, owner=data)
    ix = (slice(1, 1023),) * 3
    for axis in (None, (0,)):
        act = Active(var, resident=True)
        for _ in range(3):
            act.mean(axis=axis)
            t0 = time.perf_counter()
            act[ix]
            print("query", axis, round((time.perf_counter() - t0) * 1e3, 3), "ms", flush=True)
        act.mean(axis=axis)
        pr = cProfile.Profile()
        pr.enable()
        act[ix]
        pr.disable()
        pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
    release_resident(var)


if __name__ == "__main__":
    main()
