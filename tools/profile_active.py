"""cProfile of one Active query on the C3 file (host-side phase costs).
    python tools/profile_active.py [axis...]   e.g. python tools/profile_active.py 0 2"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tools.bench_active as B  # noqa: E402


def main():
    resident = "--resident" in sys.argv
    axis = tuple(int(x) for x in sys.argv[1:] if x != "--resident") or None
    import numpy as np
    import torch
    from pyactivestorage_amd.active import Active
    from pyactivestorage_amd.synthetic import chunk_major_device
    from pyactivestorage_amd.variable import ChunkedVariable
    n, c = 1024, 64
    shape, chunks = (n, n, n), (c, c, c)
    data, offsets, _ = chunk_major_device(torch, shape, chunks, np.float32, torch.device("cuda", 0),
                                          fill=-999.0, fill_frac=0.01)
    path = "/tmp/pyas_prof.chunks"
    with open(path, "wb") as f:
        for o in range(0, data.numel(), 256 << 20):
            f.write(data[o:o + (256 << 20)].cpu().numpy().tobytes())
    del data
    torch.cuda.empty_cache()
    grid = [s // k for s, k in zip(shape, chunks)]
    index = {cc: (int(offsets[i]), c ** 3 * 4) for i, cc in enumerate(np.ndindex(*grid))}
    attrs = {"_FillValue": np.array([-999.0], dtype=np.float32)}
    var = ChunkedVariable(name="c3", shape=shape, chunks=chunks, dtype=np.float32, chunk_index=index,
                          attrs=attrs, filename=path)
    act = Active(var, resident=resident)
    act.mean(axis=axis)
    act[...]
    act.mean(axis=axis)
    pr = cProfile.Profile()
    pr.enable()
    act[...]
    pr.disable()
    os.unlink(path)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
