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
    ap.add_argument("--gpu-only", action="store_true", help="skip the per-call and oracle legs")
    ap.add_argument("--trials", type=int, default=5, help="timed passes of the GPU leg (median reported)")
    ap.add_argument("--ceiling-read", action="store_true",
                    help="diagnostic: also time the same pool doing only the file reads "
                         "(open + pread of each chunk into a per-thread buffer, no GPU)")
    ap.add_argument("--ceiling-us", type=int, default=0,
                    help="diagnostic: also time the same pool driving a function that only "
                         "sleeps this long with the GIL released (the pattern's own ceiling)")
    ap.add_argument("--cpu-chunks", type=int, default=256)
    ap.add_argument("--percall-chunks", type=int, default=1024,
                    help="chunks timed through the per-call path (PYAS_COALESCE off)")
    ap.add_argument("--zlib", action="store_true",
                    help="store each chunk byte-shuffled + deflated (level 4), as netCDF4 files do")
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
    comp = pas.Zlib(4) if a.zlib else None
    filters = [pas.Shuffle(4)] if a.zlib else None
    rcomp = ref.Zlib(4) if a.zlib else None
    rfilters = [ref.Shuffle(4)] if a.zlib else None
    offs, sizes = [], []
    try:
        import zlib as _z
        with open(path, "wb") as f:
            pos = 0
            for k in range(a.chunks):
                x = (np.arange(c ** 3, dtype=np.float32) + k * c ** 3)
                x[rng.random(x.size) < 0.01] = -999.0
                raw = x.tobytes()
                if a.zlib:
                    raw = _z.compress(np.frombuffer(raw, np.uint8).reshape(-1, 4).T.tobytes(), 4)
                offs.append(pos)
                sizes.append(len(raw))
                f.write(raw)
                pos += len(raw)

        def run(fn, n, oracle=False, trials=1):
            def one(k):
                return fn(path, offs[k], sizes[k], rcomp if oracle else comp,
                          rfilters if oracle else filters, missing, np.dtype("<f4"), (c, c, c), "C",
                          sel, axis, np.ma.sum)
            ts = []
            for _ in range(trials):
                # a fresh pool per trial, as Active._from_storage builds one per query
                with concurrent.futures.ThreadPoolExecutor(max_workers=a.threads) as ex:
                    list(ex.map(one, range(min(n, 64))))          # warm-up
                    t0 = time.perf_counter()
                    res = list(ex.map(one, range(n)))
                    ts.append(time.perf_counter() - t0)
            return float(np.median(ts)), res

        from pyactivestorage_amd.device import get_context
        s0 = get_context(0).coalescer_stats() if pas.COALESCE else None
        c0 = os.times()
        gs, gres = run(pas.reduce_chunk, a.chunks, trials=a.trials)
        c1 = os.times()
        cpu_us = ((c1.user - c0.user) + (c1.system - c0.system)) / (a.chunks * a.trials) * 1e6
        s1 = get_context(0).coalescer_stats() if pas.COALESCE else None
        if a.gpu_only:
            extra = {}
            if a.ceiling_us:
                import ctypes
                libc = ctypes.CDLL("libc.so.6")

                def idle(*args):
                    libc.usleep(a.ceiling_us)
                    return None
                ns, _ = run(idle, a.chunks, trials=a.trials)
                extra = {"ceiling_us": a.ceiling_us, "ceiling_chunks_per_s": round(a.chunks / ns, 1)}
            if a.ceiling_read:
                import threading
                tl = threading.local()

                def read_only(p, off, size, *args):
                    b = getattr(tl, "b", None)
                    if b is None or len(b) < size:
                        b = tl.b = bytearray(size)
                    fd = os.open(p, os.O_RDONLY)
                    try:
                        os.preadv(fd, [memoryview(b)[:size]], off)
                    finally:
                        os.close(fd)
                    return None
                rs_, _ = run(read_only, a.chunks, trials=a.trials)
                extra["read_only_chunks_per_s"] = round(a.chunks / rs_, 1)
            print(json.dumps({"threads": a.threads, "chunks_per_s": round(a.chunks / gs, 1),
                              "env": {k: v for k, v in os.environ.items() if k.startswith("PYAS_")},
                              "cpu_us_per_chunk": round(cpu_us, 1),
                              "stats": {k: s1[k] - s0[k] for k in s1}, **extra}), flush=True)
            return
        ceiling = None
        if a.ceiling_read:
            import threading
            tl2 = threading.local()

            def read_only2(p, off, size, *args):
                b = getattr(tl2, "b", None)
                if b is None or len(b) < size:
                    b = tl2.b = bytearray(size)
                fd = os.open(p, os.O_RDONLY)
                try:
                    os.preadv(fd, [memoryview(b)[:size]], off)
                finally:
                    os.close(fd)
            rs2, _ = run(read_only2, a.chunks, trials=a.trials)
            ceiling = round(a.chunks / rs2, 1)
        pas.COALESCE = False
        ps, pres = run(pas.reduce_chunk, min(a.percall_chunks, a.chunks))
        pas.COALESCE = True
        cs, cres = run(ref.reduce_chunk, a.cpu_chunks, oracle=True)
        for k in range(a.cpu_chunks):               # parity of the sample
            assert int(np.asarray(gres[k][1]).reshape(-1)[0]) == int(np.asarray(cres[k][1]).reshape(-1)[0])
            np.testing.assert_allclose(np.ma.filled(gres[k][0], 0), np.ma.filled(cres[k][0], 0), rtol=1e-6)
        for k in range(min(a.percall_chunks, a.chunks)):      # both GPU paths agree
            assert np.ma.getdata(gres[k][0]).tobytes() == np.ma.getdata(pres[k][0]).tobytes()
        npc = min(a.percall_chunks, a.chunks)
        out = {"workload": f"reduce_chunk per chunk, {a.threads}-thread pool, 64^3 f32 masked sum, "
                           f"{'shuffle+zlib ' if a.zlib else ''}page-cache file (active.py:557-589 pattern)",
               "gpu": {"chunks": a.chunks, "trials": a.trials, "s_median": round(gs, 4), "chunks_per_s": round(a.chunks / gs, 1),
                       "GBps": round(a.chunks * cb / gs / 1e9, 3),
                       "path": "coalesced (pyas_coalesced_reduce)" if s1 else "per-call",
                       "batches": (s1["batches"] - s0["batches"]) if s1 else None,
                       "largest_batch": s1["largest"] if s1 else None,
                       "dispatcher_busy_s": round(s1["busy_s"] - s0["busy_s"], 4) if s1 else None,
                       "callers_read_s": round(s1["read_s"] - s0["read_s"], 4) if s1 else None,
                       "callers_wait_s": round(s1["wait_s"] - s0["wait_s"], 4) if s1 else None,
                       "host_cpu_us_per_chunk": round(cpu_us, 1)},
               "read_only_ceiling_chunks_per_s": ceiling,
               "gpu_per_call": {"chunks": npc, "s": round(ps, 4), "chunks_per_s": round(npc / ps, 1),
                                "GBps": round(npc * cb / ps / 1e9, 3)},
               "cpu_oracle": {"chunks": a.cpu_chunks, "s": round(cs, 4),
                              "chunks_per_s": round(a.cpu_chunks / cs, 1),
                              "GBps": round(a.cpu_chunks * cb / cs / 1e9, 3)}}
        print(json.dumps(out), flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)


if __name__ == "__main__":
    main()
