"""Probe: per-chunk partials of a few selections through ReductionPlan vs NumPy
(debugging aid for run_spans)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyactivestorage_amd import selection
from pyactivestorage_amd.batch import ReductionPlan
from pyactivestorage_amd.device import DeviceBuffer, get_context

ctx = get_context(0)
shape = (16, 16, 64)
rng = np.random.default_rng(1)
x = rng.uniform(1, 1000, size=shape).astype(np.float32)
sels = [
    (np.array([3]), slice(15, None, -3), slice(None)),
    (3, slice(15, None, -3), slice(None)),
    (np.array([3]), slice(0, 16, 3), slice(None)),
    (slice(3, 4), slice(0, 16, 3), slice(None)),
    (slice(3, 4), slice(15, None, -3), slice(None)),
    (np.array([3]), slice(None), slice(None)),
    (slice(None), slice(0, 16, 3), slice(None)),
    (slice(None), slice(15, None, -3), slice(None)),
    (slice(None), slice(None), slice(1, 64)),
    (slice(None), slice(None), slice(0, 63, 2)),
]
n = len(sels)
nb = x.nbytes
host = np.concatenate([np.frombuffer(x.tobytes(), np.uint8)] * n)
buf = DeviceBuffer(ctx, host.nbytes)
ctx.h2d(buf.ptr, host, None)
ctx.synchronize(None)
cs = [selection.normalize(s, shape) for s in sels]
plan = ReductionPlan(ctx, np.float32, shape, buf.ptr, np.arange(n, dtype=np.int64) * nb, selections=cs,
                     missing=(None,) * 4, round_to_var=False)
plan.launch()
parts = plan.read_chunk_partials()
for s, p in zip(sels, parts):
    w = x[s]
    print(s, "count", int(p["count"]), w.size, "min", p["min"], w.min(), "max", p["max"], w.max(),
          "sum", p["sum"], float(w.astype(np.float64).sum()))
