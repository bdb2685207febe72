"""Per-chunk drop-in throughput: the reference's own driving pattern.

``Active._from_storage`` calls ``reduce_chunk`` once per chunk from a
30-thread pool (``activestorage/active.py:557-589``), each call opening the
file and reading its chunk (``storage.py:51-53``).  This drives
:func:`pyactivestorage_amd.storage.reduce_chunk` the same way over the C3
workload (64^3 f32 chunks in a page-cache-hot chunk-major file, _FillValue +
valid_min/valid_max, np.ma.sum) and reports chunks/s and GB/s, next to the
oracle (the reference's NumPy algorithm) on the same pool for a sample.

    python tools/bench_dropin.py [--chunks 1024] [--threads 30]
"""
import argparse
import concurrent.futures
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=30)
    ap.add_argument("--cpu-chunks", type=int, default=256)
    a = ap.parse_args()
    from oracle import storage_ref as ref
    from pyactivestorage_amd import storage as pas
    c = 64
    rng = np.random.default_rng(0)
    cb = c ** 3 * 4
    path = os.path.join(tempfile.gettempdir(), f"pyas_dropin_{os.getpid()}.chunks")
    missing = (np.float32(-999.0), None, np.float32(1000.0), np.float32(5e8))
    sel = (slice(0, c, 1),) * 3
    axis = (0, 1, 2)
    try:
        with open(path, "wb") as f:
            for k in range(a.chunks):
                x = (np.arange(c ** 3, dtype=np.float32) + k * c ** 3)
                x[rng.random(x.size) < 0.01] = -999.0
                f.write(x.tobytes())

        def run(fn, n):
            def one(k):
                return fn(path, k * cb, cb, None, None, missing, np.dtype("<f4"), (c, c, c), "C",
                          sel, axis, np.ma.sum)
            with concurrent.futures.ThreadPoolExecutor(max_workers=a.threads) as ex:
                list(ex.map(one, range(min(n, 64))))          # warm-up
                t0 = time.perf_counter()
                res = list(ex.map(one, range(n)))
                return time.perf_counter() - t0, res

        gs, gres = run(pas.reduce_chunk, a.chunks)
        cs, cres = run(ref.reduce_chunk, a.cpu_chunks)
        for k in range(a.cpu_chunks):               # parity of the sample
            assert int(np.asarray(gres[k][1]).reshape(-1)[0]) == int(np.asarray(cres[k][1]).reshape(-1)[0])
            np.testing.assert_allclose(np.ma.filled(gres[k][0], 0), np.ma.filled(cres[k][0], 0), rtol=1e-6)
        out = {"workload": f"reduce_chunk per chunk, {a.threads}-thread pool, 64^3 f32 masked sum, "
                           "page-cache file (active.py:557-589 pattern)",
               "gpu": {"chunks": a.chunks, "s": round(gs, 4), "chunks_per_s": round(a.chunks / gs, 1),
                       "GBps": round(a.chunks * cb / gs / 1e9, 3)},
               "cpu_oracle": {"chunks": a.cpu_chunks, "s": round(cs, 4),
                              "chunks_per_s": round(a.cpu_chunks / cs, 1),
                              "GBps": round(a.cpu_chunks * cb / cs / 1e9, 3)}}
        print(json.dumps(out), flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)


if __name__ == "__main__":
    main()
