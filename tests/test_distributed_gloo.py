"""Multi-rank path on CPU: world_size 2 over gloo.

The GPU run shards the chunk list into contiguous ranges (one per rank),
reduces each range on its own device and exchanges the 32-byte partials with
ONE all-gather (RCCL over xGMI); the combine is a fixed rank-order fold.
Here the same sharding + exchange code runs over gloo with CPU tensors, the
per-rank partials computed by the oracle, and the result must equal the
oracle's single-process combine (``active.py:594-598`` semantics).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import storage_ref as ref
from pyactivestorage_amd import _lib
from pyactivestorage_amd.distributed import equal_ranges, exchange_partials, shard_ranges
from pyactivestorage_amd.engine import partial_dtype
from pyactivestorage_amd.synthetic import chunk_major_host

SHAPE, CHUNKS = (16, 8, 12), (4, 4, 6)
MISSING = (np.float32(5.0), None, np.float32(3.0), np.float32(900.0))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _chunk_partials(buf, lo, hi):
    """Oracle partial per chunk, rounded to the variable dtype like Active's
    out[] (active.py:512,585), packed as pyas_partial."""
    cb = int(np.prod(CHUNKS)) * 4
    out = np.zeros(hi - lo, dtype=partial_dtype("<f4"))
    for i, c in enumerate(range(lo, hi)):
        raw = buf[c * cb:(c + 1) * cb].tobytes()
        sel = (slice(None),) * 3
        s, n = ref.reduce_chunk_bytes(raw, None, None, MISSING, "<f4", CHUNKS, "C", sel, None, np.ma.sum)
        mn, _ = ref.reduce_chunk_bytes(raw, None, None, MISSING, "<f4", CHUNKS, "C", sel, None, np.ma.min)
        mx, _ = ref.reduce_chunk_bytes(raw, None, None, MISSING, "<f4", CHUNKS, "C", sel, None, np.ma.max)
        cnt = int(n.reshape(-1)[0])
        out[i]["count"] = cnt
        out[i]["sum"] = float(np.float32(np.ma.filled(s, 0).reshape(-1)[0]))
        out[i]["min"] = float(np.ma.filled(mn, 0).reshape(-1)[0])
        out[i]["max"] = float(np.ma.filled(mx, 0).reshape(-1)[0])
    return out


def _fold(parts):
    """Fixed-order combine (the semantics of k_combine, test-side on CPU)."""
    tot = np.zeros(1, dtype=parts.dtype)
    tot["sum"] = parts["sum"].sum()
    valid = parts["count"] > 0
    tot["count"] = parts["count"].sum()
    if valid.any():
        tot["min"] = parts["min"][valid].min()
        tot["max"] = parts["max"][valid].max()
    return tot


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        buf, offsets = chunk_major_host(SHAPE, CHUNKS, np.float32)
        lo, hi = equal_ranges(len(offsets), world)[rank]
        local = _fold(_chunk_partials(buf, lo, hi))
        t = torch.from_numpy(local.view(np.uint8).copy())
        gathered = exchange_partials(torch, t)
        parts = np.frombuffer(gathered.numpy().tobytes(), dtype=partial_dtype("<f4"))
        final = _fold(parts)
        q.put((rank, gathered.numel(), final.tobytes()))
    finally:
        dist.destroy_process_group()


def test_shard_ranges_balanced_and_contiguous():
    w = np.array([5, 1, 1, 1, 9, 2, 2, 3, 0, 4], dtype=float)
    for world in (1, 2, 3, 4, 7, 12):
        r = shard_ranges(w, world)
        assert len(r) == world and r[0][0] == 0 and r[-1][1] == len(w)
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        loads = [w[a:b].sum() for a, b in r]
        assert max(loads) <= w.sum() / world + w.max()
    assert equal_ranges(4096, 8) == [(i * 512, (i + 1) * 512) for i in range(8)]


def test_two_rank_gloo_exchange_matches_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buf, offsets = chunk_major_host(SHAPE, CHUNKS, np.float32)
    want = _fold(_chunk_partials(buf, 0, len(offsets)))
    for rank, n, final in res:
        assert n == world * _lib.PARTIAL_NBYTES
        got = np.frombuffer(final, dtype=partial_dtype("<f4"))
        assert got["count"][0] == want["count"][0]
        assert got["min"][0] == want["min"][0] and got["max"][0] == want["max"][0]
        assert got["sum"][0] == pytest.approx(want["sum"][0], rel=1e-12)
    # and the Active-level answer: mean over the whole variable
    data = np.ma.asarray(ref.mask_missing(buf.view(np.float32).copy(), MISSING))
    assert want["count"][0] == np.ma.count(data)
