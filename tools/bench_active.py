"""End-to-end Active queries on the C3 workload (1024^3 f32 in 64^3 chunks,
_FillValue + valid_min/valid_max): a chunk-major file in the page cache ->
Active.__getitem__ (plan, native pread ring -> H2D, fused reduce, combine)
-> masked result.  Times whole queries for the full reduction and for
partial-axis reductions (row f1 end to end, active.py:487-516,591-630).

    python tools/bench_active.py [--reps 3] [--shape 1024]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shape", type=int, default=1024)
    ap.add_argument("--zlib", action="store_true",
                    help="chunks HDF5-shuffled + deflated (level 4, as test1.nc): 32 distinct "
                         "compressed chunks repeated over the variable (rows f2+f3 end to end)")
    ap.add_argument("--axes", default="all", help="'all', 'none' (full reduction only) or one axis tuple such as '0' or '1,2'")
    ap.add_argument("--resident", action="store_true",
                    help="Active(resident=True): chunks stay in HBM; the timed queries repeat a "
                         "query whose chunks the warm-up already loaded")
    ap.add_argument("--profile", action="store_true",
                    help="cProfile three more queries per axis; print the top host functions")
    ap.add_argument("--fold-blocks", type=int, default=0,
                    help="workgroup floor of the in-kernel layer fold (0: library default)")
    a = ap.parse_args()
    import torch
    from pyactivestorage_amd.active import Active
    from pyactivestorage_amd.synthetic import chunk_major_device
    from pyactivestorage_amd.variable import ChunkedVariable
    n, c = a.shape, 64
    shape, chunks = (n, n, n), (c, c, c)
    dev = torch.device("cuda", 0)
    if a.fold_blocks:
        from pyactivestorage_amd.device import get_context
        get_context(0).set_fold_min_blocks(a.fold_blocks)
    path = os.path.join(tempfile.gettempdir(), f"pyas_active_{os.getpid()}.chunks")
    grid = [s // k for s, k in zip(shape, chunks)]
    cb = c * c * c * 4
    res = {}
    filters = None
    try:
        if a.zlib:
            from tools.bench_inflate import make_streams
            streams = [z for _, z in make_streams(32, 4)]
            index, pos = {}, 0
            with open(path, "wb") as f:
                for i, cc in enumerate(np.ndindex(*grid)):
                    z = streams[i % len(streams)]
                    f.write(z)
                    index[cc] = (pos, len(z))
                    pos += len(z)
            filters = [{"filter_id": 2, "client_data": [4]}, {"filter_id": 1, "client_data": [4]}]
        else:
            data, offsets, _ = chunk_major_device(torch, shape, chunks, np.float32, dev, fill=-999.0,
                                                  fill_frac=0.01)
            with open(path, "wb") as f:
                step = 256 << 20
                for o in range(0, data.numel(), step):
                    f.write(data[o:o + step].cpu().numpy().tobytes())
            del data
            torch.cuda.empty_cache()
            index = {cc: (int(offsets[i]), cb) for i, cc in enumerate(np.ndindex(*grid))}
        attrs = {"_FillValue": np.array([-999.0], dtype=np.float32),
                 "valid_min": np.array([1000.0], dtype=np.float32),
                 "valid_max": np.array([5e8], dtype=np.float32)}
        var = ChunkedVariable(name="c3", shape=shape, chunks=chunks, dtype=np.float32,
                              chunk_index=index, attrs=attrs, filename=path, filter_pipeline=filters)
        nbytes = n ** 3 * 4
        axes_list = (None,) if a.axes == "none" else (None, (0,), (1,), (2,), (0, 1), (1, 2), (0, 2))
        if a.axes not in ("all", "none"):     # one axis tuple, e.g. "0" or "1,2"
            axes_list = (tuple(int(x) for x in a.axes.split(",")),)
        for axis in axes_list:
            act = Active(var, resident=a.resident)
            act.mean(axis=axis)
            act[...]                       # warm-up (pinned ring, kernels)
            times = []
            for _ in range(a.reps):
                act.mean(axis=axis)
                t0 = time.perf_counter()
                r = act[...]
                times.append(time.perf_counter() - t0)
            t = float(np.median(times))
            rate = "GBps_hbm_resident_query" if a.resident else "GBps_file_to_result"
            res[str(axis)] = {"s": round(t, 4), "ms": round(t * 1e3, 3), rate: round(nbytes / t / 1e9, 2),
                              "result_shape": list(np.shape(r))}
            print(json.dumps({str(axis): res[str(axis)]}), flush=True)
            if a.profile:
                import cProfile
                import pstats
                pr = cProfile.Profile()
                pr.enable()
                for _ in range(3):
                    act.mean(axis=axis)
                    act[...]
                pr.disable()
                pstats.Stats(pr).sort_stats("tottime").print_stats(22)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    kind = ("shuffle+zlib level-4 chunks" if a.zlib else "uncompressed chunks") + \
        (", resident in HBM after the first query" if a.resident else "")
    print(json.dumps({"workload": f"Active.mean over c3 {shape} file of {kind} (page cache) -> result",
                      "results": res}))


if __name__ == "__main__":
    main()
