import os, sys, time, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from pyactivestorage_amd.active import Active
from pyactivestorage_amd.synthetic import chunk_major_device
from pyactivestorage_amd.variable import ChunkedVariable
n, c = 1024, 64
shape, chunks = (n, n, n), (c, c, c)
data, offsets, _ = chunk_major_device(torch, shape, chunks, np.float32, torch.device("cuda", 0), fill=-999.0, fill_frac=0.01)
path = "/tmp/sel_probe.chunks"
with open(path, "wb") as f:
    for o in range(0, data.numel(), 256 << 20):
        f.write(data[o:o + (256 << 20)].cpu().numpy().tobytes())
del data
grid = [s // k for s, k in zip(shape, chunks)]
index = {cc: (int(offsets[i]), c ** 3 * 4) for i, cc in enumerate(np.ndindex(*grid))}
var = ChunkedVariable(name="c3", shape=shape, chunks=chunks, dtype=np.float32, chunk_index=index,
                      attrs={"_FillValue": np.array([-999.0], np.float32)}, filename=path)
for sl in (slice(0, 64), slice(0, 256)):
    a = Active(var)
    t = time.perf_counter(); r = a[sl]; dt = time.perf_counter() - t
    print("select", sl, r.shape, "%.3f s" % dt, "%.2f GB/s" % (r.size * 4 / dt / 1e9), flush=True)
os.unlink(path)
