"""Where Active should inflate zlib chunks (row f3): on the device
(pyas_inflate, one two-wave decoder per stream) or on the host reader threads
straight into the pinned ring (pyas_read_ranges_zlib).

A chunk file of 1 MiB streams (64^3 f32, HDF5-shuffled, zlib level 4 as the
reference's test1.nc; 32 distinct streams repeated) in the page cache; for k
touched chunks, Active(...).mean over [0:64k] end to end, median of --reps,
with device_inflate=True and False.  Then the reference's own zlib files
(tests/golden/nc: test1.nc, CMIP6-test.nc) with True / False / "auto".

    python tools/bench_inflate_crossover.py [--reps 5] [--ks 1,2,4,...]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _time(fn, reps):
    fn()   # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="1,2,4,8,16,32,64,96,128,192,256,512")
    ap.add_argument("--threads", type=int, default=30, help="Active max_threads (the reference's pool)")
    a = ap.parse_args()
    from pyactivestorage_amd import active as A
    from pyactivestorage_amd.active import Active
    from pyactivestorage_amd.variable import ChunkedVariable
    from tools.bench_inflate import make_streams

    ks = [int(k) for k in a.ks.split(",")]
    kmax = max(ks)
    streams = [z for _, z in make_streams(32, 4)]
    path = os.path.join(tempfile.gettempdir(), f"pyas_xover_{os.getpid()}.chunks")
    out = {"workload": "Active.mean over k zlib chunks (1 MiB, shuffled f32, level 4) of a page-cached file",
           "threads": a.threads, "crossover_per_thread": A._INFLATE_CROSSOVER, "sweep": {}, "files": {}}
    try:
        index, pos = {}, 0
        with open(path, "wb") as f:
            for i in range(kmax):
                z = streams[i % len(streams)]
                f.write(z)
                index[(i, 0, 0)] = (pos, len(z))
                pos += len(z)
        var = ChunkedVariable(name="x", shape=(64 * kmax, 64, 64), chunks=(64, 64, 64), dtype=np.float32,
                              chunk_index=index, attrs={}, filename=path,
                              filter_pipeline=[{"filter_id": 2, "client_data": [4]},
                                               {"filter_id": 1, "client_data": [4]}])
        first = None
        for k in ks:
            row = {}
            for mode in (True, False):
                act = Active(var, device_inflate=mode, max_threads=a.threads)
                ix = (slice(0, 64 * k),)

                def q():
                    act.mean()
                    return act[ix]
                row["device_ms" if mode else "host_ms"] = round(_time(q, a.reps) * 1e3, 3)
            row["auto_device"] = A.inflate_on_device(k, a.threads, "auto")
            row["device_faster"] = row["device_ms"] <= row["host_ms"]
            if row["device_faster"] and first is None:
                first = k
            out["sweep"][k] = row
            print(json.dumps({k: row}), flush=True)
        out["measured_crossover_streams"] = first
        nc = os.path.join(ROOT, "tests", "golden", "nc")
        for fname, vname in (("test1.nc", "tas"), ("CMIP6-test.nc", "tas")):
            row = {}
            for label, mode in (("device", True), ("host", False), ("auto", "auto")):
                act = Active(os.path.join(nc, fname), vname, device_inflate=mode, max_threads=a.threads)

                def q():
                    act.mean()
                    return act[...]
                row[label + "_ms"] = round(_time(q, a.reps) * 1e3, 3)
            out["files"][fname] = row
            print(json.dumps({fname: row}), flush=True)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
