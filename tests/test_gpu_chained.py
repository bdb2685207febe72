"""The chained combine (the reduce kernel folding tiles -> chunks -> total in
its own tail, ``chained_tail`` in pyas_kernels.hpp) against the separately
launched combines (k_tiles_to_chunks + k_combine), which follow the fixed
order of ``Active._from_storage`` (``activestorage/active.py:575-598``).

Both must agree bit for bit: per-chunk partials and the total, for one and
several tiles per chunk, one and several combine groups (> 2048 chunks),
rounded (``round_to_var``) and raw sums, masked and unmasked, whole chunks
and hyperslabs, and on repeated launches (the arrival counters reset
themselves).  The count is also checked against NumPy.
"""
import numpy as np
import pytest

from pyactivestorage_amd import selection
from pyactivestorage_amd.batch import ReductionPlan
from pyactivestorage_amd.device import DeviceBuffer

pytestmark = pytest.mark.gpu

CHUNK = (8, 16, 16)          # 2048 elements
FILL, VMIN, VMAX = -999.0, 10.0, 900.0


def _variable(n_chunks, dtype, rng):
    elems = int(np.prod(CHUNK))
    if np.dtype(dtype).kind == "f":
        data = rng.uniform(0, 1000, size=(n_chunks, elems)).astype(dtype)
        data.reshape(-1)[rng.choice(data.size, data.size // 100, replace=False)] = FILL
    else:
        data = rng.integers(-500, 1000, size=(n_chunks, elems)).astype(dtype)
    return data


def _run(ctx, data, dtype, chained, tile_bytes, selections, masked, round_to_var, with_chunks, reps=3):
    ctx.set_chained_combine(chained)
    ctx.set_tile_bytes(tile_bytes)
    buf = DeviceBuffer(ctx, data.nbytes)
    ctx.h2d(buf.ptr, np.ascontiguousarray(data), None)
    ctx.synchronize(None)
    offsets = np.arange(data.shape[0], dtype=np.int64) * data.shape[1] * data.itemsize
    missing = (FILL, None, VMIN, VMAX) if masked else (None, None, None, None)
    plan = ReductionPlan(ctx, dtype, CHUNK, buf.ptr, offsets, selections=selections, missing=missing,
                         round_to_var=round_to_var)
    outs = []
    for _ in range(reps):
        plan.launch(chunk_partials=with_chunks)
        tot = plan.read_total()
        parts = plan.read_chunk_partials() if with_chunks else None
        outs.append((tot.tobytes(), None if parts is None else parts.tobytes()))
    for o in outs[1:]:
        _same(o, outs[0], "repeated launches differ (counters not reset?)")
    buf.free()
    return plan, outs[0]


def _same(a, b, what="chained != launched"):
    """Bitwise equality of (total bytes, chunk-partial bytes), reported compactly."""
    for k, (x, y) in enumerate(zip(a, b)):
        if x == y:
            continue
        if x is None or y is None:
            raise AssertionError(f"{what}: item {k} missing on one side")
        ax = np.frombuffer(x, dtype=np.uint8).reshape(-1, 32)
        ay = np.frombuffer(y, dtype=np.uint8).reshape(-1, 32)
        bad = np.nonzero((ax != ay).any(axis=1))[0]
        raise AssertionError(f"{what}: item {k}, {bad.size} of {ax.shape[0]} partials differ, "
                             f"first #{bad[0]}: {ax[bad[0]].tobytes().hex()} vs {ay[bad[0]].tobytes().hex()}")


@pytest.mark.parametrize("n_chunks", [1, 7, 2048, 5000])
@pytest.mark.parametrize("tile_bytes", [0, 1024])          # 1 tile / 8 tiles per f32 chunk
@pytest.mark.parametrize("masked", [False, True])
def test_chained_equals_launched(gpu, n_chunks, tile_bytes, masked):
    rng = np.random.default_rng(n_chunks + tile_bytes)
    data = _variable(n_chunks, "<f4", rng)
    try:
        for rtv in (True, False):
            _, a = _run(gpu, data, "<f4", True, tile_bytes, None, masked, rtv, True)
            _, b = _run(gpu, data, "<f4", False, tile_bytes, None, masked, rtv, True)
            _same(a, b)
            _, c = _run(gpu, data, "<f4", True, tile_bytes, None, masked, rtv, False)
            _same(c[:1], a[:1], "total without chunk_out differs")
        plan, _ = _run(gpu, data, "<f4", True, tile_bytes, None, masked, True, False, reps=1)
        tot = plan.read_total()
        if masked:
            keep = (data != np.float32(FILL)) & (data >= VMIN) & (data <= VMAX)
            assert int(tot["count"][0]) == int(keep.sum())
        else:
            assert int(tot["count"][0]) == data.size
    finally:
        gpu.set_chained_combine(True)
        gpu.set_tile_bytes(0)


@pytest.mark.parametrize("dtype", ["<f8", "<i4", ">i2"])
def test_chained_hyperslab(gpu, dtype):
    n = 3000
    rng = np.random.default_rng(3)
    data = _variable(n, dtype, rng)
    # the selected shape varies per chunk in dim 0 only (hyperslab boundaries)
    sels = [selection.normalize((slice(int(rng.integers(0, 4)), 8), slice(1, 15, 2), slice(0, 16)),
                                CHUNK) for _ in range(n)]
    try:
        for tb in (0, 512):
            _, a = _run(gpu, data, dtype, True, tb, sels, True, True, True)
            _, b = _run(gpu, data, dtype, False, tb, sels, True, True, True)
            _same(a, b)
    finally:
        gpu.set_chained_combine(True)
        gpu.set_tile_bytes(0)
