"""Synthetic ``dummy_data``-style variables, generated chunk-major.

The reference writes ``data[i, j, k] = i + j*n + k*n**2`` with an O(n^3)
Python loop (``activestorage/dummy_data.py:5-18``).  Here the same value
formula is evaluated vectorised, directly in chunk-major order (chunk after
chunk, each chunk C-ordered) — the layout of an HDF5 file's chunk index
walked in order, and the layout the device kernels read.
"""
from __future__ import annotations

import numpy as np


def chunk_grid(shape, chunks):
    return tuple(-(-s // c) for s, c in zip(shape, chunks))


def chunk_major_host(shape, chunks, dtype=np.float32, origin=(0, 0, 0)):
    """NumPy version (small sizes): returns (buffer uint8, offsets int64)."""
    grid = chunk_grid(shape, chunks)
    n = shape[0]
    out = []
    for ci in np.ndindex(*grid):
        idx = [np.arange(c * cs, c * cs + cs) + o for c, cs, o in zip(ci, chunks, origin)]
        i, j, k = np.meshgrid(*idx, indexing="ij")
        val = (i.astype(np.int64) + j * n + k * n * n).astype(np.float64).astype(dtype)
        out.append(val.reshape(-1))
    flat = np.concatenate(out)
    nbytes = int(np.prod(chunks)) * np.dtype(dtype).itemsize
    return flat.view(np.uint8), np.arange(len(out), dtype=np.int64) * nbytes


def chunk_major_device(torch, shape, chunks, dtype, device, origin=(0, 0, 0), n_formula=None,
                       fill=None, fill_frac=0.0, seed=0, shuffle=False):
    """Generate a 3-D variable chunk-major on the GPU with torch.

    Returns (uint8 tensor of all chunk bytes, int64 numpy offsets, n_fill).
    Values: dtype(i + j*n + k*n^2) with global indices offset by ``origin``;
    ``fill`` planted at a seeded ``fill_frac`` of positions
    (``np.random.default_rng(seed)``); ``shuffle`` stores every chunk
    HDF5-byte-shuffled (element size = itemsize).
    """
    tdt = {np.dtype("f4"): torch.float32, np.dtype("f8"): torch.float64}[np.dtype(dtype)]
    n = n_formula or shape[0]
    grid = chunk_grid(shape, chunks)
    nchunks = int(np.prod(grid))
    celems = int(np.prod(chunks))
    es = np.dtype(dtype).itemsize
    buf = torch.empty(nchunks * celems * es, dtype=torch.uint8, device=device)
    vals = buf.view(tdt).view(nchunks, *chunks)
    # generate one slab of chunks (along grid dim 0) at a time to bound temporaries
    c1, c2 = chunks[1], chunks[2]
    jj = torch.arange(c1, device=device, dtype=torch.int64).view(1, 1, c1, 1)
    kk = torch.arange(c2, device=device, dtype=torch.int64).view(1, 1, 1, c2)
    per_slab = grid[1] * grid[2]
    gj = torch.arange(grid[1], device=device, dtype=torch.int64).repeat_interleave(grid[2])
    gk = torch.arange(grid[2], device=device, dtype=torch.int64).repeat(grid[1])
    for g0 in range(grid[0]):
        ii = (torch.arange(chunks[0], device=device, dtype=torch.int64) + g0 * chunks[0]
              + origin[0]).view(1, chunks[0], 1, 1)
        j = (gj.view(-1, 1, 1, 1) * c1 + jj + origin[1])
        k = (gk.view(-1, 1, 1, 1) * c2 + kk + origin[2])
        v = ii + j * n + k * (n * n)
        vals[g0 * per_slab:(g0 + 1) * per_slab] = v.to(torch.float64).to(tdt)
    n_fill = 0
    if fill is not None and fill_frac > 0:
        rng = np.random.default_rng(seed)
        total = nchunks * celems
        n_fill = int(total * fill_frac)
        pos = torch.from_numpy(rng.integers(0, total, size=n_fill, dtype=np.int64)).to(device)
        vals.view(-1)[pos] = torch.tensor(fill, dtype=tdt, device=device)
    if shuffle and es > 1:
        b = buf.view(nchunks, celems, es)
        buf = b.transpose(1, 2).contiguous().view(-1)
    offsets = np.arange(nchunks, dtype=np.int64) * (celems * es)
    return buf, offsets, n_fill
