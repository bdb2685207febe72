"""Benchmark: device-resident masked reduce_chunk over a dummy_data-style
variable in 64^3 float32 chunks (BASELINE.json metric; configs[2] = C3).

One *step* = one pass of the hot path over one batch: every chunk of the
rank's variable is un-shuffled (if filtered), selected, masked (_FillValue,
valid_min, valid_max) and reduced to sum/count/min/max in one fused kernel,
the per-chunk partials are combined on the device, and for N > 1 the 32-byte
per-GPU partials are exchanged with one RCCL all-gather and combined in rank
order.  Those statistics give mean, max and min (C3's three methods).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GB/s + chunks/s device-resident masked reduce_chunk, f32 64³ chunks, 1–8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)

CONFIGS = {
    # name: (shape per rank, chunks, dtype, shuffle, masked, selection)
    "c2": dict(shape=(1024, 1024, 1024), chunks=(64, 64, 64), dtype="f4", shuffle=False,
               masked=False, hyperslab=None, desc="1024^3 f32, 64^3 chunks, no mask, sum"),
    "c3": dict(shape=(1024, 1024, 1024), chunks=(64, 64, 64), dtype="f4", shuffle=False,
               masked=True, hyperslab=None,
               desc="1024^3 f32, 64^3 chunks, _FillValue + valid_min/valid_max, mean/max/min"),
    "c4": dict(shape=(2048, 2048, 2048), chunks=(128, 128, 128), dtype="f4", shuffle=True,
               masked=True, hyperslab=None, desc="2048^3 f32, 128^3 chunks, shuffle + mask, sum"),
    "c5": dict(shape=(4096, 2048, 1024), chunks=(32, 32, 32), dtype="f8", shuffle=False,
               masked=True, hyperslab=16,
               desc="4096x2048x1024 f64, 32^3 chunks, hyperslab [16:-16]^3, masked mean"),
}
FILL = -999.0
VMIN = 1000.0
VMAX = 5e8


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--tile-bytes", type=int, default=0)
    p.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                   help="weak: each GPU adds its own slab of the variable (dim 0); "
                        "strong: one variable of the config's shape split across GPUs")
    p.add_argument("--cpu-chunks", type=int, default=4096,
                   help="chunks in the CPU-baseline sample (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=30)
    p.add_argument("--force-dist", action="store_true",
                   help="rehearsal: run the RCCL branch (init, all-gather, device combine) "
                        "even at world size 1 (launch under torch.distributed.run)")
    p.add_argument("--host-inclusive", type=int, default=1,
                   help="also time pinned host -> H2D -> reduce -> D2H (rank 0, N=1)")
    p.add_argument("--file-inclusive", type=int, default=1,
                   help="also time file (page cache) -> native pread ring -> H2D -> reduce -> scalar "
                        "(rank 0, N=1)")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return p.parse_args()


def chunk_selections(cfg, gshape, lo, hi):
    """Selection table (ABI layout, int32 [n, MAX_DIMS, 3]) of chunks [lo, hi)
    for configs with a hyperslab (margin m selects [m:-m] in every dim), and
    the selected elements per chunk.  None = every chunk fully selected."""
    m = cfg["hyperslab"]
    chunks = np.array(cfg["chunks"], dtype=np.int64)
    if m is None:
        return None, np.full(hi - lo, int(np.prod(chunks)), dtype=np.int64)
    from pyactivestorage_amd import _lib
    grid = np.array(gshape, dtype=np.int64) // chunks
    cid = np.arange(lo, hi, dtype=np.int64)
    ci = np.stack(np.unravel_index(cid, tuple(grid)), axis=1)          # (n, 3)
    start = np.maximum(m - ci * chunks, 0)
    stop = np.minimum(np.array(gshape) - m - ci * chunks, chunks)
    cnt = np.maximum(stop - start, 0)
    table = np.zeros((hi - lo, _lib.MAX_DIMS, 3), dtype=np.int32)
    table[:, :, 1] = 1
    table[:, :, 2] = 1
    table[:, :3, 0] = np.where(cnt > 0, start, 0)
    table[:, :3, 2] = cnt
    return table, cnt.prod(axis=1)


def cpu_baseline(cfg, host_chunks: np.ndarray, n_chunks: int, missing, threads: int):
    """Time the oracle (NumPy restatement of storage.reduce_chunk + the
    Active combine) on a page-cache-hot chunk-major file, fanned out over a
    ThreadPoolExecutor like active.py:557-572."""
    import concurrent.futures

    from oracle import storage_ref as ref
    dt = np.dtype(cfg["dtype"])
    chunk_bytes = int(np.prod(cfg["chunks"])) * dt.itemsize
    with tempfile.NamedTemporaryFile(dir="/tmp", suffix=".chunks", delete=False) as f:
        f.write(host_chunks.tobytes())
        path = f.name
    filters = [ref.Shuffle(dt.itemsize)] if cfg["shuffle"] else None
    sel = tuple(slice(0, c, 1) for c in cfg["chunks"])
    axis = (0, 1, 2)
    try:
        with open(path, "rb") as fh:  # warm the page cache
            while fh.read(1 << 26):
                pass
        t0 = time.perf_counter()
        with concurrent.futures.ThreadPoolExecutor(max_workers=threads) as ex:
            futs = [ex.submit(ref.reduce_chunk, path, c * chunk_bytes, chunk_bytes, None, filters,
                              missing, dt, cfg["chunks"], "C", sel, axis, np.ma.sum)
                    for c in range(n_chunks)]
            parts = []
            for c, fu in enumerate(futs):
                tmp, cnt = fu.result()
                parts.append((tmp, cnt, (slice(c, c + 1), slice(0, 1), slice(0, 1))))
        out = ref.combine_partials(parts, (n_chunks, 1, 1), dt, axis, "mean", components=True)
        dt_s = time.perf_counter() - t0
    finally:
        os.unlink(path)
    return dt_s, out


def host_inclusive(torch, ctx, data, cfg, dt, missing, reps=3, groups=16):
    """Host-resident variant of the same step: the chunk bytes start in pinned
    host memory, are copied H2D in `groups` slices on a copy stream while the
    compute stream reduces the previous slice, and the 32-byte result is
    copied back.  Returns (serial GB/s, overlapped GB/s)."""
    from pyactivestorage_amd import engine
    from pyactivestorage_amd.batch import ReductionPlan
    nbytes = data.numel()
    cb = int(np.prod(cfg["chunks"])) * dt.itemsize
    n = nbytes // cb
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.copy_(data, non_blocking=False)
    dev = torch.empty_like(data)
    comp = torch.cuda.current_stream()
    copy = torch.cuda.Stream()
    bounds = np.linspace(0, n, groups + 1).astype(np.int64)
    plans = [ReductionPlan(ctx, dt, cfg["chunks"], dev.data_ptr() + int(a) * cb,
                           np.arange(b - a, dtype=np.int64) * cb,
                           shuffle=dt.itemsize if cfg["shuffle"] else 0, missing=missing,
                           stream=comp.cuda_stream) for a, b in zip(bounds[:-1], bounds[1:])]
    totals = torch.empty(groups * 32, dtype=torch.uint8, device=data.device)
    final = torch.empty(32, dtype=torch.uint8, device=data.device)
    out = torch.empty(32, dtype=torch.uint8, pin_memory=True)

    def run(overlap):
        evs = []
        for g, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
            st = copy if overlap else comp
            with torch.cuda.stream(st):
                dev[a * cb:b * cb].copy_(host[a * cb:b * cb], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
            evs.append(ev)
        for g, p in enumerate(plans):
            comp.wait_event(evs[g])
            p.launch(comp.cuda_stream, chunk_partials=False)
            totals[g * 32:(g + 1) * 32].copy_(p.total_tensor(torch))
        engine.combine_partials(ctx, dt, totals.data_ptr(), groups, final.data_ptr(), False,
                                comp.cuda_stream)
        out.copy_(final, non_blocking=True)
        torch.cuda.synchronize()

    res = []
    for overlap in (False, True):
        run(overlap)
        t0 = time.perf_counter()
        for _ in range(reps):
            run(overlap)
        res.append(nbytes / ((time.perf_counter() - t0) / reps) / 1e9)
    del dev, host
    return res


def file_inclusive(torch, ctx, data, cfg, dt, missing, reps=3, threads=16):
    """POSIX bytes in, scalar out: the variable's chunks are written to a
    chunk-major file (left in the page cache), then each rep reads every
    chunk with the native pread ring (pyas_read_ranges: pinned slots copied
    H2D as they fill), reduces on the device and copies the 32-byte result
    back.  Returns (GB/s, seconds per rep)."""
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.ingest import read_ranges
    nbytes = data.numel()
    cb = int(np.prod(cfg["chunks"])) * dt.itemsize
    n = nbytes // cb
    path = os.path.join(tempfile.gettempdir(), f"pyas_bench_{os.getpid()}.chunks")
    try:
        with open(path, "wb") as f:
            step = 256 << 20
            for a in range(0, nbytes, step):
                f.write(data[a:a + step].cpu().numpy().tobytes())
        dev = torch.empty_like(data)
        st = torch.cuda.current_stream().cuda_stream
        plan = ReductionPlan(ctx, dt, cfg["chunks"], dev.data_ptr(), np.arange(n, dtype=np.int64) * cb,
                             shuffle=dt.itemsize if cfg["shuffle"] else 0, missing=missing, stream=st)
        offs = np.arange(n, dtype=np.int64) * cb
        sizes = np.full(n, cb, dtype=np.int64)

        def run():
            read_ranges(ctx, path, offs, sizes, dev.data_ptr(), offs, st, threads)
            plan.launch(st, chunk_partials=False)
            plan.read_total(st)

        run()
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        sec = (time.perf_counter() - t0) / reps
        del dev
        return nbytes / sec / 1e9, sec
    finally:
        if os.path.exists(path):
            os.unlink(path)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or args.force_dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from pyactivestorage_amd import _lib, engine
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.distributed import reduce_sharded
    from pyactivestorage_amd.device import get_context
    from pyactivestorage_amd.synthetic import chunk_major_device

    cfg = CONFIGS[args.config]
    dt = np.dtype(cfg["dtype"])
    ctx = get_context(local)
    if args.tile_bytes:
        ctx.set_tile_bytes(args.tile_bytes)
    stream = torch.cuda.current_stream().cuda_stream

    # the variable: weak scaling grows it along dim 0 with the GPU count
    gshape = list(cfg["shape"])
    if args.scaling == "weak":
        gshape[0] *= world
    gshape = tuple(gshape)
    grid = [s // c for s, c in zip(gshape, cfg["chunks"])]
    n_all = int(np.prod(grid))
    _, weights = chunk_selections(cfg, gshape, 0, n_all)
    from pyactivestorage_amd.distributed import shard_ranges
    lo, hi = shard_ranges(weights, world)[rank]
    data, offsets, n_fill = chunk_major_device(
        torch, gshape, cfg["chunks"], dt, dev, chunk_range=(lo, hi),
        fill=FILL if cfg["masked"] else None, fill_frac=0.01 if cfg["masked"] else 0.0,
        seed=rank, shuffle=cfg["shuffle"])
    torch.cuda.synchronize()
    missing = ((dt.type(FILL), None, dt.type(VMIN), dt.type(VMAX)) if cfg["masked"]
               else (None, None, None, None))
    sels, counts = chunk_selections(cfg, gshape, lo, hi)
    plan = ReductionPlan(ctx, dt, cfg["chunks"], data.data_ptr(), offsets,
                         shuffle=dt.itemsize if cfg["shuffle"] else 0, sel_table=sels,
                         missing=missing, round_to_var=True, stream=stream)
    n_chunks = plan.n_chunks
    sel_elems = int(counts.sum())
    bytes_per_launch = sel_elems * dt.itemsize
    check = None
    if not cfg["shuffle"] and sels is None:
        # independent device check of the unmasked count with plain torch ops
        tdt = torch.float32 if dt.itemsize == 4 else torch.float64
        v = data[: bytes_per_launch].view(tdt)
        ok = (v != FILL) & (v >= VMIN) & (v <= VMAX) if cfg["masked"] else torch.ones_like(v, dtype=torch.bool)
        check = {"torch_count": int(ok.sum().item())}
        del v, ok

    final = torch.zeros(_lib.PARTIAL_NBYTES, dtype=torch.uint8, device=dev)

    def step():
        if use_dist:
            reduce_sharded(torch, plan, ctx, stream, final)
        else:
            plan.launch(stream, chunk_partials=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    _lib.check(ctx.lib.pyas_timing_enable(ctx.handle, args.steps), "timing_enable")
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    import ctypes
    ms = (ctypes.c_float * args.steps)()
    nrec = ctypes.c_int32(0)
    _lib.check(ctx.lib.pyas_timing_read(ctx.handle, ms, args.steps, ctypes.byref(nrec)), "timing_read")
    kern_ms = float(np.mean(np.array(ms[: nrec.value]))) if nrec.value else float("nan")
    if use_dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms

    tot = plan.read_total(stream)[0]
    local = {"sum": float(tot["sum"]), "count": int(tot["count"]), "min": float(tot["min"]),
             "max": float(tot["max"])}
    if check is not None:
        check["kernel_count"] = local["count"]
        check["ok"] = check["torch_count"] == local["count"]
    result = local
    if use_dist:
        fin = np.frombuffer(final.cpu().numpy().tobytes(), dtype=engine.partial_dtype(dt))[0]
        result = {"sum": float(fin["sum"]), "count": int(fin["count"]), "min": float(fin["min"]),
                  "max": float(fin["max"])}

    ms_per_step = elapsed / args.steps * 1e3
    if use_dist:
        agg = torch.tensor([bytes_per_launch, n_chunks], dtype=torch.float64, device=dev)
        dist.all_reduce(agg)
        total_bytes, total_chunks = float(agg[0]), float(agg[1])
    else:
        total_bytes, total_chunks = float(bytes_per_launch), float(n_chunks)
    value = total_bytes / (elapsed / args.steps) / 1e9
    chunks_per_s = total_chunks / (elapsed / args.steps)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.traffic_file) as f:
            tr = json.load(f)
        ent = tr.get(args.config) if "config" not in tr else (tr if tr["config"] == args.config else None)
        if ent:
            traffic = ent.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    cpu = None
    if rank == 0 and world == 1 and args.cpu_chunks > 0:
        nc = min(args.cpu_chunks, n_chunks)
        cb = int(np.prod(cfg["chunks"])) * dt.itemsize
        host = data[: nc * cb].cpu().numpy()
        secs, _ = cpu_baseline(cfg, host, nc, missing, args.cpu_threads)
        ncores = len(os.sched_getaffinity(0))
        cpu = {"value": round(nc * cb / secs / 1e9, 4), "unit": "GB/s",
               "cores": min(args.cpu_threads, ncores), "kind": "port",
               "sample": f"{nc} of {n_chunks} chunks ({nc * cb / 2**20:.0f} MiB) of the same "
                         f"workload, oracle storage_ref.reduce_chunk per chunk from a page-cache-hot "
                         f"file on a {args.cpu_threads}-thread pool (active.py:557), "
                         f"{secs:.2f} s, host has {ncores} usable cores",
               "chunks_per_s": round(nc / secs, 1)}

    hostinc = None
    if rank == 0 and world == 1 and args.host_inclusive and data.numel() <= (8 << 30):
        ser, ovl = host_inclusive(torch, ctx, data, cfg, dt, missing)
        hostinc = {"serial_GBps": round(ser, 2), "overlapped_GBps": round(ovl, 2),
                   "path": "pinned host -> H2D (16 slices, copy stream) -> fused reduce "
                           "(compute stream) -> D2H 32 B"}

    fileinc = None
    if rank == 0 and world == 1 and args.file_inclusive and data.numel() <= (8 << 30):
        gbs, sec = file_inclusive(torch, ctx, data, cfg, dt, missing)
        fileinc = {"GBps": round(gbs, 2), "s_per_pass": round(sec, 4),
                   "path": "chunk-major file in page cache -> pyas_read_ranges (16 pread threads, "
                           "16 x 64 MiB pinned slots, H2D as slots fill) -> fused reduce -> D2H 32 B"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "f64" if dt.itemsize == 8 else "f32", "data": "synthetic",
            "config": {"workload": f"{args.config}: {cfg['desc']}", "variable": list(gshape),
                       "chunk_shape": list(cfg["chunks"]), "chunks_rank0": n_chunks,
                       "bytes_rank0": bytes_per_launch, "parallelism": f"chunk-shard x{world}",
                       "methods": "sum,count,min,max in one pass (mean = sum/count)"},
            "chunks_per_s": round(chunks_per_s, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel": "pyas::k_reduce",
                         "kernel_ms_avg": round(kern_ms, 5), "kernel_ms_avg_max_rank": round(kern_ms_max, 5),
                         "bytes_per_launch": bytes_per_launch},
            "cpu_baseline": cpu,
            "result": result, "check": check, "host_inclusive": hostinc,
            "file_inclusive": fileinc,
        }
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
