"""Throughput of the Reductionist-compatible server (row f4) under the
reference client's pattern: one POST /v2/{op}/ per chunk from a thread pool
(activestorage/active.py:557-589 -> reductionist.reduce_chunk,
reductionist.py:92-99), 64^3 f32 chunks, a missing_value rule, sum.
Reports requests/s and GB/s of chunk bytes served.

    python tools/bench_reductionist.py [--chunks 512] [--threads 30]
"""
import argparse
import concurrent.futures
import json
import os
import sys
import tempfile
import time

import numpy as np
import requests

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _client(url, ks, threads, cb, c):
    """One client process: `threads` threads, one keep-alive session each."""
    import threading
    local = threading.local()

    def one(k):
        s = getattr(local, "s", None)
        if s is None:
            s = local.s = requests.Session()
        body = {"interface_type": "s3", "url": "s3://bucket/var.bin", "dtype": "float32",
                "byte_order": "little", "offset": k * cb, "size": cb, "order": "C",
                "shape": [c, c, c], "missing": {"missing_value": 42.0}}
        r = s.post(url, json=body, timeout=60)
        r.raise_for_status()
        return len(r.content)

    with concurrent.futures.ThreadPoolExecutor(max_workers=threads) as ex:
        return sum(ex.map(one, ks))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=512)
    ap.add_argument("--threads", type=int, default=30)
    ap.add_argument("--workers", type=int, default=1, help="server processes (SO_REUSEPORT)")
    ap.add_argument("--client-procs", type=int, default=4)
    ap.add_argument("--inproc", action="store_true",
                    help="serve from a thread of this process (shares the GIL with the client)")
    a = ap.parse_args()
    from pyactivestorage_amd import reductionist_server as rs
    c = 64
    cb = c ** 3 * 4
    root = tempfile.mkdtemp(prefix="pyas_rs_")
    os.makedirs(os.path.join(root, "bucket"))
    path = os.path.join(root, "bucket", "var.bin")
    rng = np.random.default_rng(0)
    with open(path, "wb") as f:
        for k in range(a.chunks):
            x = rng.uniform(0, 100, c ** 3).astype("<f4")
            x[::97] = 42.0
            f.write(x.tobytes())
    proc = srv = None
    if a.inproc:
        srv = rs.ReductionistServer(root, ("127.0.0.1", 0))
        srv.start()
        base = srv.url
    else:   # the server in its own process, as a deployment runs it
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        proc = subprocess.Popen([sys.executable, "-m", "pyactivestorage_amd.reductionist_server", root,
                                 "--port", str(port), "--workers", str(a.workers)],
                                cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        base = f"http://127.0.0.1:{port}"
        for _ in range(600):
            try:
                requests.post(base + "/v0/", timeout=1)
                break
            except requests.ConnectionError:
                time.sleep(0.1)
    url = f"{base}/v2/sum/"
    try:
        # clients in their own processes (a Python client is GIL-bound too)
        import multiprocessing as mp
        procs = max(1, a.client_procs)
        ctx = mp.get_context("spawn")
        with ctx.Pool(procs) as pool:
            pool.starmap(_client, [(url, list(range(p, min(64, a.chunks), procs)),
                                    max(1, a.threads // procs), cb, c) for p in range(procs)])
            t0 = time.perf_counter()
            pool.starmap(_client, [(url, list(range(p, a.chunks, procs)),
                                    max(1, a.threads // procs), cb, c) for p in range(procs)])
            dt = time.perf_counter() - t0
    finally:
        if srv is not None:
            srv.shutdown()
            srv.server_close()
        if proc is not None:
            proc.terminate()
            proc.wait(timeout=30)
        os.unlink(path)
    print(json.dumps({"workload": f"Reductionist v2 sum requests, {a.threads} client threads in {a.client_procs} processes, "
                                  "64^3 f32 chunks, missing_value, server "
                                  + ("in-process" if a.inproc else f"{a.workers} server process(es)"),
                      "requests": a.chunks, "s": round(dt, 4),
                      "requests_per_s": round(a.chunks / dt, 1),
                      "GBps": round(a.chunks * cb / dt / 1e9, 3)}))


if __name__ == "__main__":
    main()
