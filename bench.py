"""Benchmark: device-resident masked reduce_chunk over a dummy_data-style
variable in 64^3 float32 chunks (BASELINE.json metric; configs[2] = C3).

One *step* = one pass of the hot path over one batch: every chunk of the
rank's variable is un-shuffled (if filtered), selected, masked (_FillValue,
valid_min, valid_max) and reduced to sum/count/min/max in one fused kernel,
the per-chunk partials are combined on the device, and for N > 1 the 32-byte
per-GPU partials are exchanged with one RCCL all-gather and combined in rank
order.  Those statistics give mean, max and min (C3's three methods).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]

Multi-GPU: either ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N`` (WORLD_SIZE/RANK/LOCAL_RANK from the launcher), or plain
``python bench.py --gpus N``: with no WORLD_SIZE in the environment this
process starts N rank processes itself (before anything touches the GPU) and
exits with their status.  It never runs fewer ranks than ``--gpus`` asks for.

The JSON line's headline (``value``) is C3 at the chosen scaling (weak by
default: each GPU adds a 1024^3 slab).  ``extra`` adds the two 8-GPU configs
of BASELINE.json measured at the same N, both strong scaling (one fixed
variable split over the ranks): C4 2048^3 f32 128^3 shuffled + masked
(4096 chunks, 4096/N per rank) and C5 4096x2048x1024 f64 32^3 hyperslab
masked mean (262,144 chunks).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
    # small shapes of C3 / C4 / C5 for the N-rank rehearsal tests (not bench lines)
    "t3": dict(shape=(256, 256, 256), chunks=(64, 64, 64), dtype="f4", shuffle=False,
               masked=True, hyperslab=None, desc="test: 256^3 f32, 64^3 chunks, masked"),
    "t4": dict(shape=(256, 256, 256), chunks=(128, 128, 128), dtype="f4", shuffle=True,
               masked=True, hyperslab=None, desc="test: 256^3 f32, 128^3 chunks, shuffle + mask"),
    "t5": dict(shape=(256, 128, 128), chunks=(32, 32, 32), dtype="f8", shuffle=False,
               masked=True, hyperslab=16, desc="test: 256x128x128 f64, 32^3 chunks, hyperslab, masked"),
}
FILL = -999.0
VMIN = 1000.0
VMAX = 5e8


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--tile-bytes", type=int, default=0)
    p.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                   help="weak: each GPU adds its own slab of the variable (dim 0); "
                        "strong: one variable of the config's shape split across GPUs")
    p.add_argument("--extra", default="c4,c5,c3_slab,c3_stride",
                   help="comma list of configs also measured at this N with strong scaling "
                        "(reported under 'extra'; 'none' to skip); c3_slab / c3_stride: the "
                        "reference's query shapes through Active on C3 (N=1 only)")
    p.add_argument("--extra-steps", type=int, default=20)
    p.add_argument("--cpu-chunks", type=int, default=4096,
                   help="chunks in the CPU-baseline sample (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=30)
    p.add_argument("--force-dist", action="store_true",
                   help="rehearsal: run the RCCL branch (init, all-gather, device combine) "
                        "even at world size 1 (launch under torch.distributed.run)")
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="nccl (= RCCL, one GPU per rank); gloo: the same N-rank body with the "
                        "exchange staged through host memory, ranks may share a GPU (rehearsal "
                        "of --gpus N on a smaller box)")
    p.add_argument("--host-inclusive", type=int, default=1,
                   help="also time pinned host -> H2D -> reduce -> D2H (rank 0, N=1)")
    p.add_argument("--file-inclusive", type=int, default=1,
                   help="also time file (page cache) -> native pread ring -> H2D -> reduce -> scalar "
                        "(rank 0, N=1)")
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--selftest-launch", action="store_true",
                   help="CPU-only rehearsal of the N-rank launcher (gloo, no GPU): each rank "
                        "reduces its shard of a small variable with NumPy, the partials are "
                        "all-gathered and folded in rank order, rank 0 prints the wiring")
    p.add_argument("--selftest-hang-rank", type=int, default=-1,
                   help="with --selftest-launch: this rank sleeps instead of joining the "
                        "all-gather (the launcher's wall limit must end the run)")
    p.add_argument("--selftest-fail-rank", type=int, default=-1,
                   help="with --selftest-launch: this rank exits with status 3 after joining")
    p.add_argument("--launch-timeout", type=float, default=900.0,
                   help="N > 1 launcher: wall limit in seconds for all ranks together; past it "
                        "the ranks still running are named, stopped, and the launch exits 124")
    p.add_argument("--dist-timeout", type=float, default=300.0,
                   help="seconds a collective may wait before torch.distributed aborts it "
                        "(init_process_group timeout)")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus() -> int:
    """GPUs this process may use, counted without any HIP call: the KFD
    topology in sysfs (nodes with a non-zero gpu_id), narrowed by the
    *_VISIBLE_DEVICES variables.  -1 when sysfs cannot be read."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(root):
            with open(os.path.join(root, node, "gpu_id")) as f:
                n += int(f.read().strip() or 0) != 0
    except (OSError, ValueError):
        return -1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(n: int, argv, check_devices: bool = True, timeout: float | None = 900.0) -> int:
    """Start ``n`` rank processes of this script (one per GPU) and wait.

    Runs in a process that has not touched the GPU (it counts devices from
    sysfs, :func:`visible_gpus`, and every rank checks the count again once
    its runtime is up), and starts children rather than exec'ing, so no
    GPU-initialised process is ever replaced.  Exits non-zero if fewer than
    ``n`` devices are visible: the bench never silently runs fewer ranks.
    If one rank fails the others are stopped (they would wait forever in
    the next collective), and the failing rank is named on stderr.  Past
    ``timeout`` seconds the ranks still running are named, stopped
    (SIGTERM, then SIGKILL after 10 s) and the launch returns 124."""
    if check_devices:
        have = visible_gpus()
        if have < 0:   # no KFD topology readable: the runtime's count (amdsmi; no HIP init here)
            import torch
            have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    t0 = time.monotonic()
    rc = 0
    live = dict(enumerate(procs))
    while live:
        for r, p in list(live.items()):
            code = p.poll()
            if code is None:
                continue
            del live[r]
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {r} exited with status {code}; stopping ranks "
                      f"{sorted(live)}", file=sys.stderr, flush=True)
                for q in live.values():
                    q.terminate()
        if timeout is not None and live and time.monotonic() - t0 > timeout:
            if rc == 0:
                rc = 124
                print(f"bench.py: wall limit {timeout:.0f} s passed; ranks {sorted(live)} still "
                      f"running (hung or slow), stopping them", file=sys.stderr, flush=True)
            for q in live.values():
                q.terminate()
            t_stop = time.monotonic()
            while live and time.monotonic() - t_stop < 10:
                for r, p in list(live.items()):
                    if p.poll() is not None:
                        del live[r]
                time.sleep(0.05)
            for q in live.values():
                q.kill()
            live = {}
        time.sleep(0.05)
    for p in procs:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


def selftest_launch(rank: int, world: int, hang_rank: int = -1, dist_timeout: float = 300.0,
                    fail_rank: int = -1) -> None:
    """Rank body of ``--selftest-launch`` (CPU, gloo): the sharding and the
    rank-order fold of the GPU path, with NumPy per-chunk partials.
    ``hang_rank`` sleeps instead of joining the exchange (launcher test)."""
    import datetime

    import torch
    import torch.distributed as dist

    from pyactivestorage_amd.distributed import exchange_partials, fold_partials_host, shard_ranges
    from pyactivestorage_amd.engine import partial_dtype
    from pyactivestorage_amd.synthetic import chunk_major_host

    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=dist_timeout))
    if rank == hang_rank:
        time.sleep(3600)
    if rank == fail_rank:
        sys.exit(3)
    shape, chunks = (32, 16, 24), (8, 8, 8)
    buf, offsets = chunk_major_host(shape, chunks, np.float32)
    vals = buf.view(np.float32).reshape(len(offsets), -1)
    vals = np.where(np.arange(vals.size).reshape(vals.shape) % 7 == 0, np.float32(FILL), vals)
    pdt = partial_dtype("<f4")
    parts = np.zeros(len(offsets), dtype=pdt)
    for c in range(len(offsets)):
        ok = vals[c][(vals[c] != FILL) & (vals[c] >= 3.0)]
        parts[c]["count"] = ok.size
        parts[c]["sum"] = float(ok.astype(np.float64).sum())
        parts[c]["min"] = float(ok.min()) if ok.size else 0.0
        parts[c]["max"] = float(ok.max()) if ok.size else 0.0
    lo, hi = shard_ranges(np.ones(len(offsets)), world)[rank]
    local = fold_partials_host(parts[lo:hi])
    gathered = exchange_partials(torch, torch.from_numpy(local.view(np.uint8).copy()))
    final = fold_partials_host(np.frombuffer(gathered.numpy().tobytes(), dtype=pdt))
    ranges = [None] * world
    dist.all_gather_object(ranges, {"rank": rank, "env_rank": int(os.environ["RANK"]),
                                    "local_rank": int(os.environ["LOCAL_RANK"]),
                                    "world": int(os.environ["WORLD_SIZE"]),
                                    "range": [lo, hi]})
    if rank == 0:
        single = fold_partials_host(parts)
        print(json.dumps({"selftest": "launch", "n_ranks": world, "ranks": ranges,
                          "final": {k: final[k][0].item() for k in pdt.names},
                          "single": {k: single[k][0].item() for k in pdt.names}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


# ---------------------------------------------------------------------------
# workload
# ---------------------------------------------------------------------------
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


def cpu_baseline(cfg, host_chunks: np.ndarray, n_chunks: int, missing, threads: int, check_minmax=False):
    """Time the oracle (NumPy restatement of storage.reduce_chunk + the
    Active combine) on a page-cache-hot chunk-major file, fanned out over a
    ThreadPoolExecutor like active.py:557-572.  Returns (seconds, the
    oracle's mean components {"sum", "n"}, and with ``check_minmax`` its
    min and max over the same chunks, untimed)."""
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
        if check_minmax:
            for kind, fn in (("min", np.ma.min), ("max", np.ma.max)):
                with concurrent.futures.ThreadPoolExecutor(max_workers=threads) as ex:
                    futs = [ex.submit(ref.reduce_chunk, path, c * chunk_bytes, chunk_bytes, None, filters,
                                      missing, dt, cfg["chunks"], "C", sel, axis, fn)
                            for c in range(n_chunks)]
                    mp = [(fu.result()[0], None, (slice(c, c + 1), slice(0, 1), slice(0, 1)))
                          for c, fu in enumerate(futs)]
                out[kind] = ref.combine_partials(mp, (n_chunks, 1, 1), dt, axis, kind)
    finally:
        os.unlink(path)
    return dt_s, out


def _cpu_model():
    """The host CPU's model name (/proc/cpuinfo, as lscpu reports it)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def oracle_check(gpu_result, oracle, dt):
    """The GPU's full-size result against the oracle's storage.py +
    _from_storage combine over the same chunks (active.py:575-630): count,
    min and max exact (bytes, a zero's sign included), mean within 1e-6
    relative."""
    n = int(np.asarray(oracle["n"]).reshape(-1)[0])
    osum = np.asarray(np.ma.getdata(oracle["sum"])).reshape(-1)[0]
    omean = float(osum) / n if n else float("nan")
    gmean = float(np.asarray(gpu_result["sum"], dtype=dt).astype(np.float64)) / gpu_result["count"] \
        if gpu_result["count"] else float("nan")
    rep = {"count": [gpu_result["count"], n], "mean": [gmean, omean]}
    ok = gpu_result["count"] == n and abs(gmean - omean) <= 1e-6 * abs(omean)
    for kind in ("min", "max"):
        if kind in oracle:
            ov = np.asarray(np.ma.getdata(oracle[kind])).reshape(-1)[0]
            gv = np.asarray(gpu_result[kind], dtype=dt)
            rep[kind] = [float(gv), float(ov)]
            ok = ok and gv.tobytes() == np.asarray(ov, dtype=dt).tobytes()
    rep["ok"] = bool(ok)
    rep["bar"] = "count/min/max bit-exact, mean <= 1e-6 relative"
    return rep


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


def _partials_dict(p):
    return {"sum": float(p["sum"]), "count": int(p["count"]), "min": float(p["min"]),
            "max": float(p["max"])}


def _same(a, b, rel=1e-6):
    """count/min/max exact, sum within ``rel`` (north_star's f32 bar)."""
    return (a["count"] == b["count"] and a["min"] == b["min"] and a["max"] == b["max"]
            and abs(a["sum"] - b["sum"]) <= rel * max(abs(b["sum"]), 1e-300))


def run_config(env, name, scaling, steps, warmup, args, full_check=False):
    """Build one config's data and plan on this rank, time ``steps`` steps
    (barrier + synchronize on both sides, max over ranks), then self-check
    the sharded result against the single-rank combine of all chunk
    partials.  Returns the per-config report (on every rank)."""
    torch, dist, ctx, dev, stream = env["torch"], env["dist"], env["ctx"], env["dev"], env["stream"]
    rank, world, use_dist = env["rank"], env["world"], env["use_dist"]
    coll_dev = env["coll_dev"]   # where collective tensors live (the GPU for RCCL, the host for gloo)
    from pyactivestorage_amd import _lib, engine
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.distributed import all_gather_bytes, reduce_sharded, shard_ranges
    from pyactivestorage_amd.synthetic import chunk_major_device

    cfg = CONFIGS[name]
    dt = np.dtype(cfg["dtype"])
    gshape = list(cfg["shape"])
    if scaling == "weak":
        gshape[0] *= world
    gshape = tuple(gshape)
    grid = [s // c for s, c in zip(gshape, cfg["chunks"])]
    n_all = int(np.prod(grid))
    _, weights = chunk_selections(cfg, gshape, 0, n_all)
    lo, hi = shard_ranges(weights, world)[rank]
    t_gen = time.perf_counter()
    data, offsets, n_fill = chunk_major_device(
        torch, gshape, cfg["chunks"], dt, dev, chunk_range=(lo, hi),
        fill=FILL if cfg["masked"] else None, fill_frac=0.01 if cfg["masked"] else 0.0,
        seed=0, shuffle=cfg["shuffle"])
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen
    missing = ((dt.type(FILL), None, dt.type(VMIN), dt.type(VMAX)) if cfg["masked"]
               else (None, None, None, None))
    sels, counts = chunk_selections(cfg, gshape, lo, hi)
    plan = ReductionPlan(ctx, dt, cfg["chunks"], data.data_ptr(), offsets,
                         shuffle=dt.itemsize if cfg["shuffle"] else 0, sel_table=sels,
                         missing=missing, round_to_var=True, stream=stream)
    n_chunks = plan.n_chunks
    bytes_per_launch = int(counts.sum()) * dt.itemsize

    check = None
    if full_check and not cfg["shuffle"] and sels is None:
        # independent device check of count/sum/min/max with plain torch ops
        tdt = torch.float32 if dt.itemsize == 4 else torch.float64
        v = data[: bytes_per_launch].view(tdt)
        ok = (v != FILL) & (v >= VMIN) & (v <= VMAX) if cfg["masked"] else None
        sel = v[ok] if ok is not None else v
        check = {"torch": {"count": int(sel.numel()), "sum": float(sel.sum(dtype=torch.float64)),
                           "min": float(sel.min()), "max": float(sel.max())}}
        del v, ok, sel

    final = torch.zeros(_lib.PARTIAL_NBYTES, dtype=torch.uint8, device=dev)
    ex_events = []

    def step(record=False):
        if use_dist:
            plan.launch(stream, chunk_partials=False)
            if record:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            gathered = reduce_sharded(torch, plan, ctx, stream, final, launch=False)
            if record:
                e1.record()
                ex_events.append((e0, e1))
            return gathered
        plan.launch(stream, chunk_partials=False)
        return None

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    _lib.check(ctx.lib.pyas_timing_enable(ctx.handle, steps), "timing_enable")
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(record=True)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    import ctypes
    ms = (ctypes.c_float * steps)()
    nrec = ctypes.c_int32(0)
    _lib.check(ctx.lib.pyas_timing_read(ctx.handle, ms, steps, ctypes.byref(nrec)), "timing_read")
    _lib.check(ctx.lib.pyas_timing_enable(ctx.handle, 0), "timing_disable")
    kern_ms = float(np.mean(np.array(ms[: nrec.value]))) if nrec.value else float("nan")
    ex_ms = float(np.mean([a.elapsed_time(b) for a, b in ex_events])) if ex_events else None

    # per-rank figures, gathered to every rank
    mine = [elapsed, kern_ms, ex_ms if ex_ms is not None else -1.0, float(bytes_per_launch),
            float(n_chunks), t_gen]
    if use_dist:
        t = torch.tensor(mine, dtype=torch.float64, device=coll_dev)
        allr = torch.empty(world * len(mine), dtype=torch.float64, device=coll_dev)
        dist.all_gather_into_tensor(allr, t)
        per = allr.view(world, len(mine)).cpu().numpy()
    else:
        per = np.array([mine])
    elapsed_max = float(per[:, 0].max())
    total_bytes, total_chunks = float(per[:, 3].sum()), float(per[:, 4].sum())

    # result + self-check: one more sharded step, then the single-rank
    # combine (pyas_combine_partials, variable-dtype rounding) over every
    # chunk partial of every rank in global chunk order must give the same
    # count/min/max and the sum within 1e-6
    plan.launch(stream, chunk_partials=True)
    local_total = _partials_dict(plan.read_total(stream)[0])
    if use_dist:
        reduce_sharded(torch, plan, ctx, stream, final, launch=False)
        torch.cuda.synchronize()
        result = _partials_dict(np.frombuffer(final.cpu().numpy().tobytes(),
                                              dtype=engine.partial_dtype(dt))[0])
    else:
        result = local_total
    cparts = plan.read_chunk_partials(stream)
    if use_dist:   # every rank's chunk partials (32 B each), as tensors
        cat = b"".join(all_gather_bytes(torch, cparts.tobytes(), coll_dev))
    else:
        cat = cparts.tobytes()
    selfcheck = None
    if rank == 0:
        n_tot = len(cat) // _lib.PARTIAL_NBYTES
        inp = torch.frombuffer(bytearray(cat), dtype=torch.uint8).to(dev)
        one = torch.zeros(_lib.PARTIAL_NBYTES, dtype=torch.uint8, device=dev)
        engine.combine_partials(ctx, dt, inp.data_ptr(), n_tot, one.data_ptr(), True, stream)
        torch.cuda.synchronize()
        single = _partials_dict(np.frombuffer(one.cpu().numpy().tobytes(),
                                              dtype=engine.partial_dtype(dt))[0])
        selfcheck = {"single_rank_combine": single, "chunks": n_tot, "ok": _same(result, single)}
        if check is not None:  # rank 0's own chunks
            check["kernel"] = local_total
            check["ok"] = _same(local_total, check["torch"])
        del inp, one
    del data, plan, final
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    rep = {
        "config": name, "desc": cfg["desc"], "scaling": scaling, "variable": list(gshape),
        "chunk_shape": list(cfg["chunks"]), "dtype": "f64" if dt.itemsize == 8 else "f32",
        "steps": steps, "warmup": warmup,
        "value": round(total_bytes / (elapsed_max / steps) / 1e9, 2), "unit": "GB/s",
        "ms_per_step": round(elapsed_max / steps * 1e3, 4),
        "chunks_per_s": round(total_chunks / (elapsed_max / steps), 1),
        "chunks_total": int(total_chunks), "bytes_total": int(total_bytes),
        "per_rank": {"kernel_ms": [round(float(x), 5) for x in per[:, 1]],
                     "exchange_combine_ms": ([round(float(x), 5) for x in per[:, 2]]
                                             if use_dist else None),
                     "chunks": [int(x) for x in per[:, 4]],
                     "gen_s": [round(float(x), 2) for x in per[:, 5]]},
        # k_reduce: every chunk whole, 4-/8-byte dtypes; k_reduce_u: selections (C5's hyperslab)
        "kernel": "pyas::k_reduce" if sels is None and dt.itemsize >= 4 else "pyas::k_reduce_u",
        "kernel_ms_rank0": round(kern_ms, 5),
        "bytes_rank0": bytes_per_launch, "chunks_rank0": n_chunks,
        "frac_rank0": round(achieved / HBM_PEAK_GBS, 4),
        "frac_min_rank": round(float((per[:, 3] / (per[:, 1] * 1e-3) / 1e9).min()) / HBM_PEAK_GBS, 4),
        "result": result, "selfcheck": selfcheck, "check": check,
    }
    return rep, achieved


# The reference's own query shapes at C3 size (tests/unit/test_active_axis.py:30-39:
# ragged hyperslabs, strides and index lists x axis subsets), each an
# Active.__getitem__ on resident chunks (active.py:487-516 -> storage.py:95).
def _list64():
    return np.sort(np.random.default_rng(7).choice(1024, size=64, replace=False))


ACTIVE_EXTRAS = {
    # name: [(label, index builder, axis, method)]
    "c3_slab": [
        ("[1:1023]^3", lambda: (slice(1, 1023),) * 3, None, "mean"),
        ("[1:1023]^3", lambda: (slice(1, 1023),) * 3, None, "min"),
        ("[0:1023]^3", lambda: (slice(0, 1023),) * 3, None, "mean"),
        ("[4:1020]^3", lambda: (slice(4, 1020),) * 3, None, "mean"),
        ("[1:1023]^3", lambda: (slice(1, 1023),) * 3, (0,), "mean"),
        ("[1:1023]^3", lambda: (slice(1, 1023),) * 3, (2,), "mean"),
        ("[1:1023]^3", lambda: (slice(1, 1023),) * 3, (0,), "min"),
        ("[1:1023]^3", lambda: (slice(1, 1023),) * 3, (2,), "min"),
    ],
    # the whole variable (zero-sign cost studies: tools/query_c3.py --zeros)
    "c3_whole": [
        ("[:]^3", lambda: (slice(None),) * 3, None, "min"),
        ("[:]^3", lambda: (slice(None),) * 3, (0,), "min"),
        ("[:]^3", lambda: (slice(None),) * 3, (2,), "min"),
    ],
    "c3_stride": [
        ("[:, 0:1024:3, :]", lambda: (slice(None), slice(0, 1024, 3), slice(None)), None, "mean"),
        ("[:, :, 0:1024:4]", lambda: (slice(None), slice(None), slice(0, 1024, 4)), None, "mean"),
        ("[:, list64, :]", lambda: (slice(None), _list64(), slice(None)), None, "mean"),
        ("[:, 0:1024:3, :]", lambda: (slice(None), slice(0, 1024, 3), slice(None)), (0,), "mean"),
        ("[:, :, 0:1024:4]", lambda: (slice(None), slice(None), slice(0, 1024, 4)), (1,), "mean"),
    ],
}


def _dim_indices(ix, n):
    """Selected indices of one dim (slice or index array), sorted unique."""
    if isinstance(ix, slice):
        return np.arange(n)[ix]
    return np.unique(np.asarray(ix))


def selected_and_touched(index, shape, chunks, es, line=128):
    """Selected bytes of an orthogonal index, and the bytes of the 128-B
    lines they touch (chunk rows line-aligned: the innermost chunk extent
    times the itemsize is a multiple of `line`)."""
    per = [_dim_indices(ix, n) for ix, n in zip(index, shape)]
    sel = int(np.prod([len(p) for p in per])) * es
    rows = int(np.prod([len(p) for p in per[:-1]]))
    inner, ci = per[-1], chunks[-1]
    assert (ci * es) % line == 0
    lines = len(np.unique((inner // ci) * (ci * es // line) + (inner % ci) * es // line))
    return sel, rows * lines * line


def run_active_extra(env, name, steps, warmup):
    """The reference's query shapes on C3 (ACTIVE_EXTRAS[name]): an
    ``Active(resident=True)`` query per step over the C3 variable held in HBM
    (attach_resident: no file), timed end to end (planning, launches, the
    combine, the result copy; the repeated query replays its cached plan).
    ``frac`` is on the selected bytes; for strides also on the touched
    128-B lines (the bytes HBM must deliver)."""
    torch, dev, rank = env["torch"], env["dev"], env["rank"]
    from pyactivestorage_amd.active import Active, attach_resident, release_resident
    from pyactivestorage_amd.synthetic import chunk_major_device
    from pyactivestorage_amd.variable import ChunkedVariable
    cfg = CONFIGS["c3"]
    dt = np.dtype(cfg["dtype"])
    shape, chunks = cfg["shape"], cfg["chunks"]
    data, offsets, _ = chunk_major_device(torch, shape, chunks, dt, dev, fill=FILL, fill_frac=0.01,
                                          seed=0, shuffle=False)
    torch.cuda.synchronize()
    grid = [s // c for s, c in zip(shape, chunks)]
    cb = int(np.prod(chunks)) * dt.itemsize
    index = {co: (int(offsets[k]), cb) for k, co in enumerate(np.ndindex(*grid))}
    attrs = {"_FillValue": np.array([FILL], dtype=dt), "valid_min": np.array([VMIN], dtype=dt),
             "valid_max": np.array([VMAX], dtype=dt)}
    var = ChunkedVariable(name=name, shape=shape, chunks=chunks, dtype=dt, chunk_index=index, attrs=attrs,
                          filename=None, filter_pipeline=None)
    attach_resident(var, data.data_ptr(), device=dev.index or 0, owner=data)
    out = []
    try:
        for label, mk, axis, method in ACTIVE_EXTRAS[name]:
            ix = mk()
            act = Active(var, resident=True, device=dev.index or 0)
            for _ in range(max(warmup, 1)):
                getattr(act, method)(axis=axis)   # a query's method lasts one __getitem__
                act[ix]
            times = []
            for _ in range(steps):
                getattr(act, method)(axis=axis)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                act[ix]
                times.append(time.perf_counter() - t0)
            ms = float(np.median(times)) * 1e3
            sel, touched = selected_and_touched(ix, shape, chunks, dt.itemsize)
            rep = {"index": label, "axis": list(axis) if axis else None, "method": method,
                   "ms_per_step": round(ms, 4), "ms_min": round(min(times) * 1e3, 4),
                   "selected_bytes": sel, "GBps": round(sel / (ms * 1e-3) / 1e9, 1),
                   "frac": round(sel / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
            if touched != sel:
                rep["touched_line_bytes"] = touched
                rep["frac_touched_lines"] = round(touched / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            out.append(rep)
    finally:
        release_resident(var)
        del data
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return {"config": name, "workload": "Active(resident) queries over C3 (1024^3 f32, 64^3 chunks, "
                                        "_FillValue + valid_min/valid_max), end to end per query",
            "steps": steps, "queries": out,
            "frac_basis": "selected bytes / median query time / 8 TB/s; strides also on the 128-B "
                          "lines they touch"}


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # plain `python bench.py --gpus N`: become the launcher of N ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:],
                              check_devices=not args.selftest_launch and args.dist_backend == "nccl",
                              timeout=args.launch_timeout if args.launch_timeout > 0 else None))
    world = int(world_env or 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.selftest_launch:
        selftest_launch(rank, world, args.selftest_hang_rank, args.dist_timeout, args.selftest_fail_rank)
        return

    import torch
    import torch.distributed as dist

    use_dist = world > 1 or args.force_dist
    ndev = torch.cuda.device_count()
    gloo = args.dist_backend == "gloo"
    if not gloo and ndev < world:   # each rank checks the launcher's sysfs count
        print(f"bench.py: rank {rank}: WORLD_SIZE {world} but {ndev} GPU(s) visible", file=sys.stderr)
        sys.exit(2)
    gpu = local % max(ndev, 1) if gloo else local   # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if use_dist:
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a bounded timeout: a rank stuck in a collective aborts with an error
        # instead of hanging the whole run (torch's nccl watchdog enforces it)
        limit = datetime.timedelta(seconds=args.dist_timeout)
        if gloo:
            dist.init_process_group("gloo", timeout=limit)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=limit)

    from pyactivestorage_amd.device import get_context

    ctx = get_context(gpu)
    if args.tile_bytes:
        ctx.set_tile_bytes(args.tile_bytes)
    env = dict(torch=torch, dist=dist, ctx=ctx, dev=dev, stream=torch.cuda.current_stream().cuda_stream,
               rank=rank, world=world, use_dist=use_dist,
               coll_dev=torch.device("cpu") if gloo else dev)

    cfg = CONFIGS[args.config]
    dt = np.dtype(cfg["dtype"])
    head, achieved = run_config(env, args.config, args.scaling, args.steps, args.warmup, args,
                                full_check=True)

    traffic = None
    try:
        with open(args.traffic_file) as f:
            tr = json.load(f)
        ent = tr.get(args.config) if "config" not in tr else (tr if tr["config"] == args.config else None)
        if ent:
            traffic = ent.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    # CPU baseline and host/file-inclusive legs: rank 0 at N=1 only
    cpu = hostinc = fileinc = ocheck = None
    if rank == 0 and world == 1 and (args.cpu_chunks > 0 or args.host_inclusive or args.file_inclusive):
        from pyactivestorage_amd.synthetic import chunk_major_device
        data, _, _ = chunk_major_device(torch, cfg["shape"], cfg["chunks"], dt, dev,
                                        fill=FILL if cfg["masked"] else None,
                                        fill_frac=0.01 if cfg["masked"] else 0.0, seed=0,
                                        shuffle=cfg["shuffle"])
        missing = ((dt.type(FILL), None, dt.type(VMIN), dt.type(VMAX)) if cfg["masked"]
                   else (None, None, None, None))
        n_chunks = head["chunks_rank0"]
        cb = int(np.prod(cfg["chunks"])) * dt.itemsize
        if args.cpu_chunks > 0:
            nc = min(args.cpu_chunks, n_chunks)
            host = data[: nc * cb].cpu().numpy()
            full = nc == n_chunks and args.scaling == "weak" and cfg["hyperslab"] is None
            secs, oracle = cpu_baseline(cfg, host, nc, missing, args.cpu_threads, check_minmax=full)
            if full:   # the GPU's full-size result against the oracle's (not timed)
                ocheck = oracle_check(head["result"], oracle, dt)
                ocheck["chunks"] = nc
            ncores = len(os.sched_getaffinity(0))
            cpu = {"value": round(nc * cb / secs / 1e9, 4), "unit": "GB/s",
                   "cores": min(args.cpu_threads, ncores), "kind": "port",
                   "sample": f"{nc} of {n_chunks} chunks ({nc * cb / 2**20:.0f} MiB) of the same "
                             f"workload, oracle storage_ref.reduce_chunk per chunk from a page-cache-hot "
                             f"file on a {args.cpu_threads}-thread pool (active.py:557), "
                             f"{secs:.2f} s; 'cores' = pool threads used, the host has {ncores} "
                             f"usable cores",
                   "chunks_per_s": round(nc / secs, 1), "cpu_model": _cpu_model()}
            del host
        if args.host_inclusive and data.numel() <= (8 << 30):
            ser, ovl = host_inclusive(torch, ctx, data, cfg, dt, missing)
            hostinc = {"serial_GBps": round(ser, 2), "overlapped_GBps": round(ovl, 2),
                       "path": "pinned host -> H2D (16 slices, copy stream) -> fused reduce "
                               "(compute stream) -> D2H 32 B"}
        if args.file_inclusive and data.numel() <= (8 << 30):
            gbs, sec = file_inclusive(torch, ctx, data, cfg, dt, missing)
            fileinc = {"GBps": round(gbs, 2), "s_per_pass": round(sec, 4),
                       "path": "chunk-major file in page cache -> pyas_read_ranges (16 pread threads, "
                               "16 x 64 MiB pinned slots, H2D as slots fill) -> fused reduce -> D2H 32 B"}
        del data
        torch.cuda.empty_cache()

    extra = {}
    names = [] if args.extra in ("", "none") else [c.strip() for c in args.extra.split(",")]
    for name in names:
        if name in ACTIVE_EXTRAS:
            if world == 1:   # single-GPU query shapes (the N-rank curve is the head + C4/C5)
                extra[name] = run_active_extra(env, name, args.extra_steps, args.warmup)
            continue
        if name not in CONFIGS:
            raise SystemExit(f"bench.py: unknown --extra config {name!r}")
        rep, _ = run_config(env, name, "strong", args.extra_steps, args.warmup, args)
        rep.pop("check", None)
        extra[f"{name}_strong"] = rep

    if rank == 0:
        line = {
            "metric": METRIC, "value": head["value"], "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": head["dtype"], "data": "synthetic",
            "config": {"workload": f"{args.config}: {cfg['desc']}", "variable": head["variable"],
                       "exchange": (args.dist_backend if use_dist else None),
                       "chunk_shape": head["chunk_shape"], "chunks_total": head["chunks_total"],
                       "chunks_rank0": head["chunks_rank0"], "bytes_rank0": head["bytes_rank0"],
                       "parallelism": f"chunk-shard x{world}",
                       "methods": "sum,count,min,max in one pass (mean = sum/count)"},
            "chunks_per_s": head["chunks_per_s"],
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": "profile figure, not measured in this run: profiles/traffic.json "
                                           "(rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes of this config's "
                                           "k_reduce, per launch)",
                         "kernel": head["kernel"], "kernel_ms_avg": head["kernel_ms_rank0"],
                         "bytes_per_launch": head["bytes_rank0"]},
            "per_rank": head["per_rank"],
            "cpu_baseline": cpu,
            "oracle_check": ocheck,
            "result": head["result"], "check": head["check"], "selfcheck": head["selfcheck"],
            "host_inclusive": hostinc, "file_inclusive": fileinc,
            "extra": extra or None,
        }
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
