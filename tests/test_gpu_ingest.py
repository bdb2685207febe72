"""Row f2: native file ingest (``pyas_read_ranges``) against the reader path.

The reference reads every chunk with its own ``open`` + ``read_block``
(``activestorage/storage.py:51-53,156-162``).  Here the golden chunks of the
reference's test files are written back at their original byte offsets into
a sparse temp file, and ``Active`` over that file (native pread ring -> pinned
slots -> H2D, then device inflate for zlib chunks) must return exactly what
``Active`` over the in-memory reader returns, which the reference's own
known answers already pin (tests/test_gpu_active.py).  Also: large ranges
that span several staging slots, tiny slots (ring wrap-around), and the
reference's error types for a missing file and a truncated one.
"""
import os

import numpy as np
import pytest

from pyactivestorage_amd import ingest
from pyactivestorage_amd.active import Active
from pyactivestorage_amd.device import DeviceBuffer
from tests import _golden as G
from tests.test_gpu_active import variable

pytestmark = pytest.mark.gpu

KEYS = ["test1.nc:tas", "cesm2_native.nc:TREFHT", "daily_data_masked.nc:ta", "CMIP6-test.nc:tas"]


def _file_variable(key, tmp_path):
    v = variable(key)
    meta, blobs = G.h5_meta()[key], G.h5_blobs()[key]
    path = tmp_path / (key.replace(":", "_") + ".bin")
    with open(path, "wb") as f:
        for ch in meta["chunk_table"]:
            f.seek(ch["offset"])
            f.write(blobs[ch["blob_start"]: ch["blob_start"] + ch["size"]].tobytes())
    v.reader = None
    v.filename = str(path)
    return v


@pytest.mark.parametrize("key", KEYS)
def test_active_file_equals_reader(gpu, key, tmp_path):
    fv = _file_variable(key, tmp_path)
    mv = variable(key)
    for method in ("mean", "min", "max", "sum"):
        for axis in (None, (0,), (1, 2)):
            a, b = Active(fv, axis=axis), Active(mv, axis=axis)
            a.method = b.method = method
            x, y = a[...], b[...]
            assert x.dtype == y.dtype and x.shape == y.shape
            np.testing.assert_array_equal(np.ma.getmaskarray(x), np.ma.getmaskarray(y))
            np.testing.assert_array_equal(np.ma.filled(x, 0), np.ma.filled(y, 0))
            assert a.data_read == b.data_read


@pytest.mark.parametrize("slots,slot_bytes", [(16, 64 << 20), (2, 1 << 16), (3, 100_000)])
def test_read_ranges_roundtrip(gpu, tmp_path, slots, slot_bytes):
    """Random ranges (some larger than a slot, some empty) land byte-exact."""
    rng = np.random.default_rng(slots)
    blob = rng.integers(0, 256, size=6 << 20, dtype=np.uint8)
    path = tmp_path / "blob.bin"
    blob.tofile(path)
    n = 200
    sizes = rng.integers(0, 300_000, size=n).astype(np.int64)
    sizes[::17] = 0
    sizes[5] = 2_500_000
    foff = np.array([rng.integers(0, blob.size - s + 1) for s in sizes], dtype=np.int64)
    doff = np.concatenate([[0], np.cumsum(-(-sizes // 256) * 256)[:-1]]).astype(np.int64)
    total = int(doff[-1] + sizes[-1])
    try:
        ingest.set_slots(gpu, slots, slot_bytes)
        dev = DeviceBuffer(gpu, max(total, 1))
        st = gpu.thread_stream()
        for threads in (1, 7):
            assert ingest.read_ranges(gpu, str(path), foff, sizes, dev.ptr, doff, st, threads) == sizes.sum()
            host = np.zeros(max(total, 1), dtype=np.uint8)
            gpu.d2h(host, dev.ptr, st)
            for i in range(n):
                np.testing.assert_array_equal(host[doff[i]: doff[i] + sizes[i]],
                                              blob[foff[i]: foff[i] + sizes[i]])
    finally:
        ingest.set_slots(gpu, 16, 64 << 20)


def test_read_ranges_errors(gpu, tmp_path):
    path = tmp_path / "short.bin"
    path.write_bytes(b"x" * 1000)
    dev = DeviceBuffer(gpu, 4096)
    st = gpu.thread_stream()
    with pytest.raises(FileNotFoundError):           # storage.py:51 open(rfile)
        ingest.read_ranges(gpu, str(tmp_path / "missing.bin"), [0], [10], dev.ptr, [0], st)
    with pytest.raises(OSError, match="short read"):
        ingest.read_ranges(gpu, str(path), [0, 900], [10, 200], dev.ptr, [0, 16], st)
    with pytest.raises(ValueError):
        ingest.read_ranges(gpu, str(path), [0, 1], [10], dev.ptr, [0], st)
    # the context still works after a failed read
    assert ingest.read_ranges(gpu, str(path), [10], [20], dev.ptr, [0], st) == 20


def test_truncated_chunk_file(gpu, tmp_path):
    """A chunk index pointing past the end of the file fails like a short read."""
    fv = _file_variable("cesm2_native.nc:TREFHT", tmp_path)
    size = os.path.getsize(fv.filename)
    with open(fv.filename, "r+b") as f:
        f.truncate(size - 100)
    a = Active(fv)
    a.method = "mean"
    with pytest.raises(OSError):
        a[...]


def test_read_ranges_zlib(gpu, tmp_path):
    """pyas_read_ranges_zlib (host inflate into the pinned ring, row f3 below
    the crossover): the bytes zlib.decompress gives (storage.py:119-120),
    zlib's own error for a broken stream, and the reference's reshape
    ValueError for a stream of the wrong inflated size."""
    import zlib
    rng = np.random.default_rng(4)
    chunk = 4096
    plains = [np.cumsum(rng.normal(size=chunk // 4)).astype("<f4").tobytes() for _ in range(40)]
    comps = [zlib.compress(p, int(lvl)) for p, lvl in zip(plains, rng.integers(0, 10, len(plains)))]
    path = tmp_path / "z.bin"
    blob = b"".join(comps)
    path.write_bytes(blob)
    foff = np.concatenate([[0], np.cumsum([len(c) for c in comps])[:-1]]).astype(np.int64)
    size = np.array([len(c) for c in comps], dtype=np.int64)
    stride = 4096 + 256
    doff = np.arange(len(comps), dtype=np.int64) * stride
    dev = DeviceBuffer(gpu, len(comps) * stride)
    st = gpu.thread_stream()
    for threads in (1, 4, 30):
        assert ingest.read_ranges_zlib(gpu, str(path), foff, size, dev.ptr, doff, chunk, st, threads) == size.sum()
        host = np.zeros(len(comps) * stride, dtype=np.uint8)
        gpu.d2h(host, dev.ptr, st)
        gpu.synchronize(st)
        for k, p in enumerate(plains):
            assert host[k * stride: k * stride + chunk].tobytes() == p, (threads, k)
    bad = bytearray(blob)
    bad[foff[7] + 20] ^= 0xFF                        # corrupt one stream's compressed bytes
    bpath = tmp_path / "bad.bin"
    bpath.write_bytes(bytes(bad))
    try:
        zlib.decompress(bytes(bad[foff[7]: foff[7] + size[7]]))
        broken = False
    except zlib.error:
        broken = True
    if broken:
        with pytest.raises(zlib.error):
            ingest.read_ranges_zlib(gpu, str(bpath), foff, size, dev.ptr, doff, chunk, st, 4)
    big = DeviceBuffer(gpu, len(comps) * 8448)       # room for 8192 inflated bytes per stream
    with pytest.raises(ValueError, match="cannot reshape"):   # inflates to 4096, not 8192
        ingest.read_ranges_zlib(gpu, str(path), foff, size, big.ptr, doff // stride * 8448, 8192, st, 4,
                                reshape=(4, (2048,)))
    # the context still works after the failures
    assert ingest.read_ranges_zlib(gpu, str(path), foff[:3], size[:3], dev.ptr, doff[:3], chunk, st) == size[:3].sum()
