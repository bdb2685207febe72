"""Throughput of pyas_unshuffle_chunks (the resident store's batched
un-shuffle): 4096 x 1 MiB chunks (C3 size), element size 4 and 8, device to
device.  Reports ms per launch and the HBM rate counting read + write."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pyactivestorage_amd import engine
    from pyactivestorage_amd.device import DeviceBuffer, get_context
    ctx = get_context(0)
    st = ctx.thread_stream()
    n, nbytes = 4096, 1 << 20
    src, dst = DeviceBuffer(ctx, n * nbytes), DeviceBuffer(ctx, n * nbytes)
    offs = np.arange(n, dtype=np.int64) * nbytes
    meta = DeviceBuffer(ctx, 16 * n)
    ctx.h2d(meta.ptr, np.concatenate([offs, offs[::-1].copy()]), st)
    res = {}
    for es in (2, 4, 8):
        for _ in range(3):
            engine.unshuffle_chunks(ctx, src.ptr, meta.ptr, dst.ptr, meta.ptr + 8 * n, n, nbytes, es, st)
        ctx.synchronize(st)
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            engine.unshuffle_chunks(ctx, src.ptr, meta.ptr, dst.ptr, meta.ptr + 8 * n, n, nbytes, es, st)
        ctx.synchronize(st)
        dt = (time.perf_counter() - t0) / reps
        res[f"es{es}"] = {"ms": round(dt * 1e3, 3), "GBps_read_plus_write": round(2 * n * nbytes / dt / 1e9, 1)}
    print(json.dumps({"workload": "pyas_unshuffle_chunks, 4096 x 1 MiB chunks", "results": res}))


if __name__ == "__main__":
    main()
