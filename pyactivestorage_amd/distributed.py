"""Multi-GPU sharding of a chunk reduction: one process per GPU.

The reference's only parallelism is a thread pool over chunks
(``activestorage/active.py:557-572``); chunks are independent and the combine
(``active.py:594-598``) is associative.  Here the chunk list of a query is
split into contiguous ranges, one per rank (balanced by selected elements);
each rank reduces its range from its own HBM in one launch chain, and the
ranks exchange their 32-byte partial ``{sum, count, min, max}`` with ONE
collective — an all-gather over RCCL (xGMI), 32·N bytes in total — followed
by a fixed rank-order combine on the device, so the result does not depend
on arrival order and equals the single-GPU combine order for the same
sharding.  The message is latency-bound (~10 µs), not bandwidth-bound.
"""
from __future__ import annotations

import numpy as np

from . import _lib, engine


def shard_ranges(weights, world: int):
    """Split chunks 0..n-1 into ``world`` contiguous ranges of near-equal total
    weight (selected elements per chunk).  Returns a list of (lo, hi)."""
    w = np.asarray(weights, dtype=np.float64).reshape(-1)
    n = w.size
    if world < 1:
        raise ValueError("world must be >= 1")
    if n == 0:
        return [(0, 0)] * world
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(cum, target, side="left"))
        k = min(max(k, cuts[-1]), n)
        cuts.append(k)
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def equal_ranges(n_chunks: int, world: int):
    return shard_ranges(np.ones(n_chunks), world)


def fold_partials_host(parts: np.ndarray) -> np.ndarray:
    """Host statement of the rank-order fold (``k_combine``'s semantics on
    a handful of 32-byte partials): sums added in order, counts added,
    min/max over partials with count > 0.  Used where no device is present
    (the CPU launcher rehearsal); the GPU path folds with
    :func:`device_combine`."""
    tot = np.zeros(1, dtype=parts.dtype)
    s = parts["sum"].dtype.type(0)
    for v in parts["sum"]:
        s = s + v
    tot["sum"] = s
    tot["count"] = parts["count"].sum()
    valid = parts["count"] > 0
    if valid.any():
        tot["min"] = parts["min"][valid].min()
        tot["max"] = parts["max"][valid].max()
    return tot


def exchange_partials(torch, local_total, group=None):
    """All-gather the 32-byte per-rank partial (uint8 tensor) over the
    process group (RCCL for CUDA tensors, gloo for CPU tensors).  Returns a
    (world * 32,) uint8 tensor in rank order."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    src = local_total.reshape(-1)
    staged = dist.get_backend(group) == "gloo" and src.device.type != "cpu"
    if staged:   # gloo moves host memory: stage the 32 bytes through it
        src = src.cpu()
    out = torch.empty(world * _lib.PARTIAL_NBYTES, dtype=torch.uint8, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.to(local_total.device) if staged else out


def all_gather_bytes(torch, data: bytes, device, group=None) -> list:
    """All-gather one variable-length byte string per rank as tensors (two
    collectives: the lengths, then the payloads padded to the longest);
    returns the ranks' strings in rank order.  ``device``: where the
    tensors live (the GPU for RCCL, the host for gloo)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([len(data)], dtype=torch.int64, device=device)
    lens = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(lens, n, group=group)
    lens = [int(x) for x in lens.cpu()]
    m = max(max(lens), 1)
    buf = torch.zeros(m, dtype=torch.uint8)
    if data:
        buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    buf = buf.to(device)
    out = torch.empty(world * m, dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, buf, group=group)
    host = out.cpu().numpy()
    return [host[r * m: r * m + lens[r]].tobytes() for r in range(world)]


def device_combine(ctx, dtype, gathered, out, stream):
    """Fixed rank-order combine of gathered partials on the GPU (HIP kernel).
    Per-chunk rounding to the variable dtype already happened on each rank."""
    world = gathered.numel() // _lib.PARTIAL_NBYTES
    engine.combine_partials(ctx, dtype, gathered.data_ptr(), world, out.data_ptr(), False, stream)


def reduce_sharded(torch, plan, ctx, stream, final, group=None, combine=None, launch=True):
    """One sharded step: local fused reduce -> RCCL all-gather -> combine.

    ``plan`` is this rank's :class:`~pyactivestorage_amd.batch.ReductionPlan`
    over its chunk range; ``final`` a 32-byte uint8 device tensor that
    receives the global partial.  ``combine`` defaults to the device kernel.
    ``launch=False`` skips the local reduce (the caller already queued it).
    """
    if launch:
        plan.launch(stream, chunk_partials=False)
    local = plan.total_tensor(torch)
    gathered = exchange_partials(torch, local, group)
    (combine or device_combine)(ctx, plan.dtype, gathered, final, stream)
    return gathered
