"""Zero-heavy min/max queries: the cost of NumPy's zero sign.

A C3-sized variable (1024^3 f32 in 64^3 chunks, _FillValue -999 only) where
a fraction of the elements are +0.0 or -0.0 (random signs) and the rest are
positive, so the min of every chunk, and of nearly every partial-axis
output, is a zero: the shape of a precipitation or sea-ice field.  The
variable is written as a chunk-major file and queried through
``Active(resident=True)``, so the timed queries read HBM only.  Each query
is timed end to end (median of --reps); run under ``rocprofv3
--kernel-trace --stats`` for the per-kernel split (reduce vs the pyas_tie_*
passes).  ``--zeros 0`` makes the same variable without zeros (the tie
passes then return at once): the difference is the tie cost.

    python tools/bench_zeros.py [--zeros 0.5] [--axes none,0,2] [--reps 10]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("PYAS_TREE"):   # A/B: another build of the package (e.g. the previous round's)
    sys.path.insert(0, os.environ["PYAS_TREE"])


def make_variable(torch, path, n, c, zeros, seed=0):
    """Write the chunk-major file; returns the chunk index."""
    grid = (n // c,) * 3
    celems = c ** 3
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    index = {}
    per = 64            # chunks generated per batch
    coords = list(np.ndindex(*grid))
    with open(path, "wb") as f:
        for b0 in range(0, len(coords), per):
            nb = min(per, len(coords) - b0)
            u = torch.rand(nb * celems, generator=g, device="cuda")
            v = 1.0 + torch.rand(nb * celems, generator=g, device="cuda") * 999.0
            if zeros > 0:
                sgn = torch.rand(nb * celems, generator=g, device="cuda") < 0.5
                z = torch.where(sgn, torch.tensor(-0.0, device="cuda"), torch.tensor(0.0, device="cuda"))
                v = torch.where(u < zeros, z, v)
            f.write(v.cpu().numpy().astype(np.float32).tobytes())
            for i in range(nb):
                index[coords[b0 + i]] = ((b0 + i) * celems * 4, celems * 4)
    return index


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, default=1024)
    ap.add_argument("--zeros", type=float, default=0.5, help="fraction of elements that are +-0.0")
    ap.add_argument("--axes", default="none,0,2", help="comma list of 'none' or one axis (0/1/2)")
    ap.add_argument("--method", default="min")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--index", default="",
                    help="a hyperslab, e.g. '1:1023' for every dim (cuts the edge chunks: the "
                         "two-step path and its zero-sign passes instead of the fold)")
    a = ap.parse_args()
    import torch
    from pyactivestorage_amd.active import Active, release_resident
    from pyactivestorage_amd.variable import ChunkedVariable
    n, c = a.shape, 64
    path = os.path.join(tempfile.gettempdir(), f"pyas_zeros_{os.getpid()}.chunks")
    res = {}
    try:
        index = make_variable(torch, path, n, c, a.zeros)
        attrs = {"_FillValue": np.array([-999.0], dtype=np.float32)}
        var = ChunkedVariable(name="zeros", shape=(n,) * 3, chunks=(c,) * 3, dtype=np.float32,
                              chunk_index=index, attrs=attrs, filename=path, filter_pipeline=None)
        index = Ellipsis
        if a.index:
            lo, hi = (int(x) for x in a.index.split(":"))
            index = (slice(lo, hi),) * 3
        for ax in a.axes.split(","):
            axis = None if ax == "none" else (int(ax),)
            act = Active(var, resident=True)
            getattr(act, a.method)(axis=axis)
            r = act[index]                  # loads the chunks into HBM
            act[index]
            times = []
            for _ in range(a.reps):
                getattr(act, a.method)(axis=axis)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = act[index]
                times.append(time.perf_counter() - t0)
            arr = np.ma.getdata(r)
            zero = arr == 0
            res[ax] = {"ms": round(float(np.median(times)) * 1e3, 3), "ms_min": round(min(times) * 1e3, 3),
                       "outputs": int(arr.size), "zero_outputs": int(zero.sum()),
                       "negative_zero_outputs": int((zero & np.signbit(arr)).sum())}
            print(json.dumps({ax: res[ax]}), flush=True)
        release_resident(var)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    print(json.dumps({"workload": f"Active({a.method}, resident) over {n}^3 f32, 64^3 chunks"
                                  f"{', index [' + a.index + ']^3' if a.index else ''}, "
                                  f"{a.zeros:.0%} of elements +-0.0, rest in [1, 1000)",
                      "results": res}))


if __name__ == "__main__":
    main()
