"""The predicate stream of cut chunks (``run_spans`` in pyas_kernels.hpp)
against the oracle, chunk by chunk.

``run_spans`` reads a chunk's selection as spans (the selected index tuples
of the outer dims) of aligned 16-B groups with a per-lane predicate, so a
cut chunk of a hyperslab, a strided or a listed selection is streamed like a
whole one.  Its hazards are the group geometry: spans that start off a 16-B
boundary (chunk offsets that are only element-aligned, cuts at any index),
rows whose length is not a multiple of the group, strided innermost dims,
negative steps, index lists in the outer dims, shuffled chunks (16-element
groups over the byte planes), and span-granular tiling (several tiles per
chunk, fewer spans than tiles).  Every case here compares each chunk's
partial (sum, count, min, max) of a ``ReductionPlan`` batch with
``oracle.storage_ref.reduce_chunk_bytes`` (``storage.py:95-100``) on the
same bytes: count/min/max exact, sums within the north-star 1e-6.
"""
import zlib

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import selection
from pyactivestorage_amd.batch import ReductionPlan
from pyactivestorage_amd.device import DeviceBuffer
from tests._compare import shuffle_bytes

pytestmark = pytest.mark.gpu

FILL, VMIN, VMAX = 77, 5, 900


def _dim_sel(rng, n):
    """One dim of a chunk selection: whole, cut run, strided (either sign),
    an index list, or an integer."""
    r = rng.integers(0, 10)
    if r < 2:
        return slice(None)
    if r < 5:                                   # a cut run (the hyperslab edge)
        a = int(rng.integers(0, max(1, n // 3)))
        b = int(rng.integers(max(a + 1, 2 * n // 3), n + 1))
        return slice(a, b)
    if r < 7:                                   # strided
        s = int(rng.integers(2, 5))
        a = int(rng.integers(0, min(3, n)))
        return slice(a, n, s) if rng.integers(0, 2) else slice(n - 1 - a, None, -s)
    if r < 9:                                   # sorted index list
        k = int(rng.integers(1, min(6, n) + 1))
        return np.sort(rng.choice(n, size=k, replace=False))
    return int(rng.integers(0, n))


def _selections(rng, shape, n):
    sels = []
    for c in range(n):
        if c % 5 == 0:   # the shapes hyperslab edges produce: one or two dims cut at either end
            sel = [slice(None)] * len(shape)
            for d in rng.choice(len(shape), size=int(rng.integers(1, min(2, len(shape)) + 1)), replace=False):
                m = shape[d]
                sel[d] = slice(int(rng.integers(1, m // 2 + 1)), None) if rng.integers(0, 2) else \
                    slice(0, int(rng.integers(m // 2, m)))
            sels.append(tuple(sel))
        else:
            sel = [_dim_sel(rng, m) for m in shape]
            lists = [d for d, x in enumerate(sel) if isinstance(x, np.ndarray)]
            for d in lists[1:]:        # one index list per selection (NumPy's orthogonal case)
                sel[d] = slice(None)
            if all(isinstance(x, int) for x in sel):
                sel[0] = slice(None)   # keep one axis: a 0-d chunk[sel] has no axis to reduce
            sels.append(tuple(sel))
    return sels


def _data(dt, shape, n, rng):
    if dt.kind == "f":
        a = rng.uniform(1, 1000, size=(n,) + shape).astype(dt)
        a.reshape(-1)[::13] = FILL
    else:
        info = np.iinfo(dt)
        a = rng.integers(max(info.min, -300) if info.min < 0 else 1, min(info.max, 1000),
                         size=(n,) + shape, endpoint=True).astype(dt)
        a.reshape(-1)[::13] = FILL
    return a


CASES = [
    ("<f4", (16, 16, 64)), (">f4", (9, 10, 37)), ("<f8", (8, 12, 32)), ("<f4", (5, 6, 7, 20)),
    ("<i2", (12, 10, 48)), ("u1", (10, 9, 70)), ("<i8", (6, 7, 9)), ("<u4", (130,)),
]


@pytest.mark.parametrize("dt,shape", CASES, ids=[f"{d}-{'x'.join(map(str, s))}" for d, s in CASES])
@pytest.mark.parametrize("shuffle", [False, True])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("tile_bytes", [0, 512])
@pytest.mark.parametrize("spans", ["1", "2"])
def test_spans_match_oracle(gpu, monkeypatch, dt, shape, shuffle, masked, tile_bytes, spans):
    # PYAS_SPANS=2: aligned runs (run_rows' chunks) through run_spans too
    monkeypatch.setenv("PYAS_SPANS", spans)
    dt = np.dtype(dt)
    if shuffle and dt.itemsize == 1:
        pytest.skip("shuffle is the identity for 1-byte types")
    seed = zlib.crc32(repr((dt.str, shape, shuffle, masked, tile_bytes)).encode())
    rng = np.random.default_rng(seed)
    n = 40
    data = _data(dt, shape, n, rng)
    sels = _selections(rng, shape, n)
    nbytes = int(np.prod(shape)) * dt.itemsize
    # chunk slots only element-aligned (a 3-element pad): spans start at every
    # offset from a 16-B boundary
    slot = nbytes + 3 * dt.itemsize
    offsets = np.arange(n, dtype=np.int64) * slot + dt.itemsize
    host = np.zeros(n * slot + 64, dtype=np.uint8)
    raws = []
    for c in range(n):
        raw = data[c].tobytes()
        raws.append(raw)
        stored = shuffle_bytes(data[c], dt.itemsize) if shuffle else raw
        host[offsets[c]:offsets[c] + nbytes] = np.frombuffer(stored, dtype=np.uint8)
    missing = (FILL, None, VMIN, VMAX) if masked else (None, None, None, None)
    gpu.set_tile_bytes(tile_bytes)
    buf = DeviceBuffer(gpu, host.nbytes)
    try:
        gpu.h2d(buf.ptr, host, None)
        gpu.synchronize(None)
        cs = [selection.normalize(s, shape) for s in sels]
        plan = ReductionPlan(gpu, dt, shape, buf.ptr, offsets, shuffle=dt.itemsize if shuffle else 0,
                             selections=cs, missing=missing, round_to_var=False)
        plan.launch()
        parts = plan.read_chunk_partials()
    finally:
        gpu.set_tile_bytes(0)
        buf.free()
    for c in range(n):
        what = f"chunk {c} sel {sels[c]}"
        axis = tuple(range(len(cs[c].shape)))        # every dim of chunk[sel]
        s_w, n_w = ref.reduce_chunk_bytes(raws[c], None, None, missing, dt.str, shape, "C", sels[c],
                                          axis, np.ma.sum)
        cnt = int(np.asarray(n_w).reshape(-1)[0])
        assert int(parts[c]["count"]) == cnt, f"{what}: count {parts[c]['count']} != {cnt}"
        if cnt == 0:
            continue
        mn, _ = ref.reduce_chunk_bytes(raws[c], None, None, missing, dt.str, shape, "C", sels[c],
                                       axis, np.ma.min)
        mx, _ = ref.reduce_chunk_bytes(raws[c], None, None, missing, dt.str, shape, "C", sels[c],
                                       axis, np.ma.max)
        assert parts[c]["min"] == np.asarray(mn).reshape(-1)[0], f"{what}: min {parts[c]['min']} != {mn}"
        assert parts[c]["max"] == np.asarray(mx).reshape(-1)[0], f"{what}: max {parts[c]['max']} != {mx}"
        want = np.asarray(np.ma.getdata(s_w)).reshape(-1)[0]
        if dt.kind == "f":
            sel_abs = np.abs(data[c][sels[c]].astype(np.float64)).sum()
            assert abs(float(parts[c]["sum"]) - float(want)) <= max(1e-6 * abs(float(want)), 4e-7 * sel_abs), \
                f"{what}: sum {parts[c]['sum']} != {want}"
        else:
            assert int(parts[c]["sum"]) == int(want), f"{what}: sum {parts[c]['sum']} != {want}"
