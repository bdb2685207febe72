"""Host-cost profile of the per-chunk drop-in (single thread, then a pool).

Serial: wall time per ``reduce_chunk`` call split into the coalescer's own
phases (file read, wait for the batch) and the rest (Python + GIL), plus a
cProfile of the Python side.  Then the same calls from a pool, timing each
call's phases from the worker's point of view.
"""
import concurrent.futures
import cProfile
import json
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pyactivestorage_amd import storage as pas
    from pyactivestorage_amd.device import get_context
    c = 64
    cb = c ** 3 * 4
    path = f"/tmp/pyas_prof_dropin_{os.getpid()}.chunks"
    with open(path, "wb") as f:
        for k in range(256):
            f.write((np.arange(c ** 3, dtype=np.float32) + k).tobytes())
    missing = (np.float32(-999.0), None, np.float32(1000.0), np.float32(5e8))
    sel = (slice(0, c, 1),) * 3
    dt = np.dtype("<f4")
    shape = (c, c, c)
    axis = (0, 1, 2)

    def one(k):
        return pas.reduce_chunk(path, (k % 256) * cb, cb, None, None, missing, dt, shape, "C",
                                sel, axis, np.ma.sum)
    out = {}
    for k in range(64):
        one(k)
    ctx = get_context(0)
    n = 2000
    s0 = ctx.coalescer_stats()
    t0 = time.perf_counter()
    c0 = os.times()
    for k in range(n):
        one(k)
    c1 = os.times()
    wall = time.perf_counter() - t0
    s1 = ctx.coalescer_stats()
    out["serial"] = {"us_per_call": round(wall / n * 1e6, 1),
                     "read_us": round((s1["read_s"] - s0["read_s"]) / n * 1e6, 1),
                     "wait_us": round((s1["wait_s"] - s0["wait_s"]) / n * 1e6, 1),
                     "dispatcher_busy_us": round((s1["busy_s"] - s0["busy_s"]) / n * 1e6, 1),
                     "cpu_us": round(((c1.user - c0.user) + (c1.system - c0.system)) / n * 1e6, 1)}
    pr = cProfile.Profile()
    pr.enable()
    for k in range(500):
        one(k)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime")
    top = []
    for (fn, line, name), (cc, nc, tt, ct, callers) in sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:12]:
        top.append(f"{os.path.basename(fn)}:{line}({name}) {tt / nc * 1e6:.1f}us x{nc}")
    out["serial_profile_tottime"] = top

    # pool: per-call phases as a worker sees them
    for threads in (4, 30):
        lat = []

        def timed(k):
            a = time.perf_counter()
            r = one(k)
            lat.append(time.perf_counter() - a)
            return r
        with concurrent.futures.ThreadPoolExecutor(threads) as ex:
            list(ex.map(timed, range(64)))
            lat.clear()
            s0 = ctx.coalescer_stats()
            t0 = time.perf_counter()
            list(ex.map(timed, range(4096)))
            wall = time.perf_counter() - t0
            s1 = ctx.coalescer_stats()
        m = 4096
        out[f"pool{threads}"] = {"chunks_per_s": round(m / wall, 1),
                                 "call_us_mean": round(float(np.mean(lat)) * 1e6, 1),
                                 "call_us_p50": round(float(np.median(lat)) * 1e6, 1),
                                 "read_us": round((s1["read_s"] - s0["read_s"]) / m * 1e6, 1),
                                 "wait_us": round((s1["wait_s"] - s0["wait_s"]) / m * 1e6, 1),
                                 "batch": round(m / max(1, s1["batches"] - s0["batches"]), 2)}
    os.unlink(path)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
