"""GPU zlib inflate throughput (row f3) on C3-shaped chunks.

1 MiB chunks (64^3 f32) of a smooth random field, HDF5-shuffled (es=4) and
deflated at level 4 as the reference's test1.nc is (filter client_data [4]).
32 distinct streams are replicated to `--chunks` streams (decode work does not
depend on repetition).  Reports decompressed GB/s of pyas_inflate (HIP events
on its stream) and, for context, host zlib.decompress with a thread pool.
"""
import argparse
import concurrent.futures
import json
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("PYAS_TREE"):   # A/B: another build of the package (e.g. the previous round's)
    sys.path.insert(0, os.environ["PYAS_TREE"])


def make_streams(n_unique, level, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for u in range(n_unique):
        i, j, k = np.meshgrid(*(np.arange(64, dtype=np.float32),) * 3, indexing="ij")
        f = 250.0 + 30.0 * np.sin(i / 9.0 + u) * np.cos(j / 13.0) + 0.05 * k
        f = (f + rng.normal(scale=0.5, size=f.shape)).astype(np.float32)
        sh = np.frombuffer(f.tobytes(), dtype=np.uint8).reshape(-1, 4).T.copy().tobytes()
        out.append((sh, zlib.compress(sh, level)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=2048)
    ap.add_argument("--level", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host zlib pool size (0: every core this process may run on, os.sched_getaffinity)")
    ap.add_argument("--wbits", type=int, default=13, help="LDS history ring (13-15)")
    ap.add_argument("--no-check", action="store_true", help="timing experiments: skip status/output checks")
    ap.add_argument("--sweep", default="", help="comma list of stream counts: per-stream rate vs streams in flight")
    args = ap.parse_args()
    if args.cpu_threads <= 0:
        args.cpu_threads = len(os.sched_getaffinity(0))
    import torch
    from pyactivestorage_amd.device import DeviceBuffer, get_context
    from pyactivestorage_amd.inflate import InflateBatch, pack_streams

    uniq = make_streams(32, args.level)
    plain_n = len(uniq[0][0])
    comps = [uniq[c % len(uniq)][1] for c in range(args.chunks)]
    host, soffs, ssizes = pack_streams(comps)
    ctx = get_context(0)
    ctx.lib.pyas_ctx_set_inflate_window_bits(ctx.handle, args.wbits)
    stream = torch.cuda.Stream()
    st = stream.cuda_stream
    src = DeviceBuffer(ctx, host.nbytes)
    dst = DeviceBuffer(ctx, args.chunks * plain_n)
    ctx.h2d(src.ptr, host, st)
    ib = InflateBatch(ctx, soffs, ssizes, np.arange(args.chunks, dtype=np.int64) * plain_n,
                      np.full(args.chunks, plain_n, dtype=np.int64))
    ib.launch(src.ptr, dst.ptr, st)
    if not args.no_check:
        ib.check(st)
        out = np.zeros(plain_n, dtype=np.uint8)
        ctx.d2h(out, dst.ptr + (args.chunks - 1) * plain_n, st)
        ctx.synchronize(st)
        assert out.tobytes() == uniq[(args.chunks - 1) % len(uniq)][0]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(args.reps):
        e0.record(stream)
        ib.launch(src.ptr, dst.ptr, st)
        e1.record(stream)
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    t0 = time.perf_counter()
    ib.launch(src.ptr, dst.ptr, st)
    ctx.synchronize(st)
    wall_ms = (time.perf_counter() - t0) * 1e3
    ms = float(np.median(times))
    total_plain = args.chunks * plain_n
    sweep = {}
    for n in [int(x) for x in args.sweep.split(",") if x]:
        n = min(n, args.chunks)
        sb = InflateBatch(ctx, soffs[:n], ssizes[:n], np.arange(n, dtype=np.int64) * plain_n,
                          np.full(n, plain_n, dtype=np.int64))
        sb.launch(src.ptr, dst.ptr, st)
        if not args.no_check:
            sb.check(st)
        ts = []
        for _ in range(args.reps):
            e0.record(stream)
            sb.launch(src.ptr, dst.ptr, st)
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        m = float(np.median(ts))
        sweep[n] = {"ms": round(m, 3), "GBps": round(n * plain_n / m / 1e6, 2),
                    "MBps_per_stream": round(plain_n / m / 1e3, 1)}
    # host zlib for context (bounded sample)
    sample = comps[: min(len(comps), 256)]
    t0 = time.perf_counter()
    with concurrent.futures.ThreadPoolExecutor(args.cpu_threads) as ex:
        list(ex.map(zlib.decompress, sample))
    cpu_s = time.perf_counter() - t0
    print(json.dumps({
        "workload": f"inflate {args.chunks} x 1 MiB shuffled f32 chunks, zlib level {args.level}",
        "ratio": round(total_plain / float(ssizes.sum()), 3),
        "gpu_ms": round(ms, 3),
        "wall_ms": round(wall_ms, 3),
        "gpu_GBps_decompressed": round(total_plain / ms / 1e6, 1),
        "gpu_GBps_compressed": round(float(ssizes.sum()) / ms / 1e6, 1),
        "cpu_GBps_decompressed": round(len(sample) * plain_n / cpu_s / 1e9, 2),
        "cpu_threads": args.cpu_threads,
        "wbits": args.wbits,
        "sweep": sweep,
    }))


if __name__ == "__main__":
    main()
