"""Synthetic ``dummy_data``-style variables, generated chunk-major.

The reference writes ``data[i, j, k] = i + j*n + k*n**2`` with an O(n^3)
Python loop (``activestorage/dummy_data.py:5-18``).  Here the same value
formula is evaluated vectorised, directly in chunk-major order (chunk after
chunk in C order of the chunk grid, each chunk C-ordered) — the layout of an
HDF5 chunk index walked in order, and the layout the device kernels read.
A contiguous range of chunks can be generated on its own, which is how each
rank of a sharded run materialises only its own part of the variable.
"""
from __future__ import annotations

import numpy as np

FILL_BLOCK = 64  # chunks per independently seeded fill-planting block


def chunk_grid(shape, chunks):
    return tuple(-(-s // c) for s, c in zip(shape, chunks))


def chunk_major_host(shape, chunks, dtype=np.float32):
    """NumPy version for small variables: (uint8 buffer, int64 offsets)."""
    if any(s % c for s, c in zip(shape, chunks)):
        raise ValueError("shape must be a multiple of the chunk shape")
    grid = chunk_grid(shape, chunks)
    n = shape[0]
    parts = []
    for ci in np.ndindex(*grid):
        idx = [np.arange(c * cs, c * cs + cs, dtype=np.int64) for c, cs in zip(ci, chunks)]
        i, j, k = np.meshgrid(*idx, indexing="ij")
        parts.append((i + j * n + k * n * n).astype(np.float64).astype(dtype).reshape(-1))
    flat = np.concatenate(parts)
    nbytes = int(np.prod(chunks)) * np.dtype(dtype).itemsize
    return flat.view(np.uint8), np.arange(len(parts), dtype=np.int64) * nbytes


def chunk_major_device(torch, shape, chunks, dtype, device, chunk_range=None, fill=None,
                       fill_frac=0.0, seed=0, shuffle=False, max_batch_bytes=1 << 29):
    """Generate chunks [lo, hi) of a 3-D variable on the GPU with torch.

    Returns (uint8 tensor of the chunks' bytes, int64 offsets into it,
    number of fill plantings).  Values: dtype(i + j*n + k*n^2) with global
    indices, n = shape[0]; ``fill`` planted at a seeded ``fill_frac`` of the
    positions (``np.random.default_rng(seed)``); ``shuffle`` stores every
    chunk HDF5-byte-shuffled (element size = itemsize).
    """
    if len(shape) != 3 or any(s % c for s, c in zip(shape, chunks)):
        raise ValueError("3-D shape that is a multiple of the chunk shape required")
    dt = np.dtype(dtype)
    tdt = {np.dtype("f4"): torch.float32, np.dtype("f8"): torch.float64}[dt]
    grid = chunk_grid(shape, chunks)
    nchunks_all = int(np.prod(grid))
    lo, hi = chunk_range if chunk_range is not None else (0, nchunks_all)
    nch = hi - lo
    celems = int(np.prod(chunks))
    es = dt.itemsize
    n = shape[0]
    buf = torch.empty(max(nch, 1) * celems * es, dtype=torch.uint8, device=device)
    vals = buf.view(tdt)[: nch * celems].view(nch, *chunks) if nch else None
    c0, c1, c2 = chunks
    ii = torch.arange(c0, device=device, dtype=torch.int64).view(1, c0, 1, 1)
    jj = torch.arange(c1, device=device, dtype=torch.int64).view(1, 1, c1, 1)
    kk = torch.arange(c2, device=device, dtype=torch.int64).view(1, 1, 1, c2)
    batch = max(1, max_batch_bytes // (celems * 8))
    for b0 in range(0, nch, batch):
        b1 = min(nch, b0 + batch)
        cid = torch.arange(lo + b0, lo + b1, device=device, dtype=torch.int64)
        g0 = cid // (grid[1] * grid[2])
        g1 = (cid // grid[2]) % grid[1]
        g2 = cid % grid[2]
        v = ((g0.view(-1, 1, 1, 1) * c0 + ii) + (g1.view(-1, 1, 1, 1) * c1 + jj) * n
             + (g2.view(-1, 1, 1, 1) * c2 + kk) * (n * n))
        vals[b0:b1] = v.to(torch.float64).to(tdt)
    n_fill = 0
    if fill is not None and fill_frac > 0 and nch:
        # planted per block of FILL_BLOCK chunks, seeded by (seed, global block
        # index): a chunk's bytes do not depend on how the chunk list is
        # sharded, so a strong-scaling run at any N reduces the same variable
        fv = torch.tensor(fill, dtype=tdt, device=device)
        flat = vals.view(-1)
        per = int(FILL_BLOCK * celems * fill_frac)
        for blk in range(lo // FILL_BLOCK, -(-hi // FILL_BLOCK)):
            rng = np.random.default_rng([seed, blk])
            pos = rng.integers(0, FILL_BLOCK * celems, size=per, dtype=np.int64)
            pos += (blk * FILL_BLOCK - lo) * celems
            pos = pos[(pos >= 0) & (pos < nch * celems)]
            n_fill += pos.size
            flat[torch.from_numpy(pos).to(device)] = fv
    if shuffle and es > 1 and nch:
        for b0 in range(0, nch, batch):  # in place, batch by batch
            b1 = min(nch, b0 + batch)
            seg = buf[b0 * celems * es: b1 * celems * es].view(b1 - b0, celems, es)
            seg.copy_(seg.transpose(1, 2).contiguous().view(b1 - b0, celems, es))
    offsets = np.arange(nch, dtype=np.int64) * (celems * es)
    return buf, offsets, n_fill
