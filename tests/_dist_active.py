"""Shared pieces of the distributed-Active GPU test (tests/test_gpu_distributed_active.py):
a synthetic chunked variable and the queries, plus the worker entry point
(run as ``python tests/_dist_active.py OUT.npz`` under RANK/WORLD_SIZE)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SHAPE, CHUNKS = (40, 36, 50), (8, 12, 10)
# (method, index, axis)
QUERIES = [
    ("mean", (slice(None),) * 3, None),
    ("sum", (slice(3, 37), slice(5, 30, 2), slice(None)), (0,)),
    ("max", (slice(3, 37), slice(5, 30, 2), slice(None)), (2,)),
    ("min", (slice(None), slice(None), slice(7, 45)), (0, 2)),
    ("mean", ([1, 5, 20, 33], slice(None), slice(10, 40)), (1,)),
    ("sum", (slice(0, 8), slice(0, 12), slice(0, 10)), None),      # a single chunk
]
# min/max of data holding both signed zeros: the result's zero sign must be
# NumPy's over the whole `out` array (zero-sign keys gathered with the grids)
ZQUERIES = [
    ("min", (slice(None),) * 3, None),
    ("min", (slice(3, 37), slice(5, 30, 2), slice(None)), (0,)),
    ("min", (slice(None), slice(None), slice(7, 45)), (1, 2)),
    ("min", (slice(None),) * 3, (0, 2)),
    ("max", (slice(None),) * 3, None),
    ("max", (slice(3, 37), slice(None), slice(None)), (2,)),
]


def make_variable(zeros=0):
    """zeros = 0: the plain variable; +1 / -1: values >= 0 / <= 0 with 20 %
    signed zeros (min / max outputs are zeros)."""
    from pyactivestorage_amd.variable import ChunkedVariable
    rng = np.random.default_rng(3 + zeros)
    a = rng.uniform(0, 100, size=SHAPE).astype("<f4")
    if zeros:
        a *= zeros
        z = rng.random(a.size) < 0.2
        a.reshape(-1)[z] = np.where(rng.random(int(z.sum())) < 0.5, -0.0, 0.0)
    a.reshape(-1)[::17] = -999.0
    grid = [s // c for s, c in zip(SHAPE, CHUNKS)]
    blobs, index, pos = [], {}, 0
    for cc in np.ndindex(*grid):
        sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(cc, CHUNKS))
        b = np.ascontiguousarray(a[sl]).tobytes()
        index[cc] = (pos, len(b))
        blobs.append(b)
        pos += len(b)
    data = b"".join(blobs)
    attrs = {"_FillValue": np.array([-999.0], dtype="<f4")}
    if not zeros:
        attrs["valid_max"] = np.array([95.0], dtype="<f4")
    return ChunkedVariable(name="v", shape=SHAPE, chunks=CHUNKS, dtype="<f4", chunk_index=index,
                           attrs=attrs, reader=lambda off, size: data[off:off + size])


def run_queries(group=None):
    from pyactivestorage_amd.active import Active
    var = make_variable()
    out = {}
    for k, (method, index, axis) in enumerate(QUERIES):
        act = Active(var, group=group)
        getattr(act, method if method != "sum" else "mean")(axis=axis)
        if method == "sum":
            act.method = "sum"
        r = act[index]
        out[f"q{k}_data"] = np.ma.getdata(r)
        out[f"q{k}_mask"] = np.ma.getmaskarray(r)
    zvar = {"min": make_variable(1), "max": make_variable(-1)}
    for k, (method, index, axis) in enumerate(ZQUERIES):
        act = Active(zvar[method], axis=axis, group=group)
        act.method = method
        r = act[index]
        out[f"z{k}_data"] = np.ma.getdata(r)
        out[f"z{k}_mask"] = np.ma.getmaskarray(r)
    return out


def main(path):
    import torch  # noqa: F401  (torch before the HIP library: one runtime)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    res = run_queries(group=dist.group.WORLD)
    if dist.get_rank() == 0:
        np.savez(path, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
