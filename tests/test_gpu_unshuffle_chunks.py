"""pyas_unshuffle_chunks (the batched device un-shuffle resident variables
use) against the oracle's restatement of numcodecs' Shuffle.decode
(``oracle/storage_ref.py:unshuffle``, call site ``storage.py:121-122``),
byte for byte: element sizes 2/4/8, chunk sizes with and without a
``n % 4`` element tail and trailing ``nbytes % es`` bytes, dword-aligned and
misaligned chunk offsets, and a scatter to non-contiguous destinations."""
import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd import engine
from pyactivestorage_amd.device import DeviceBuffer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("es", [2, 4, 8])
@pytest.mark.parametrize("nbytes", [4096, 1048576, 1000, 4096 + 3, 8 * 7])
@pytest.mark.parametrize("misalign", [0, 1, 4])
def test_unshuffle_chunks_matches_oracle(gpu, es, nbytes, misalign):
    ctx = gpu
    st = ctx.thread_stream()
    rng = np.random.default_rng(es * 1000 + nbytes + misalign)
    n = 5
    chunks = [rng.integers(0, 256, size=nbytes, dtype=np.uint8) for _ in range(n)]
    sstride = nbytes + 64 + misalign
    src = np.zeros(n * sstride + 64, dtype=np.uint8)
    soff = np.array([k * sstride + misalign for k in range(n)], dtype=np.int64)
    for k, c in enumerate(chunks):
        src[soff[k]:soff[k] + nbytes] = c
    # destinations in reverse order with gaps
    dstride = nbytes + 128
    doff = np.array([(n - 1 - k) * dstride + 16 for k in range(n)], dtype=np.int64)
    dsize = n * dstride + 64
    sbuf, dbuf = DeviceBuffer(ctx, src.nbytes), DeviceBuffer(ctx, dsize)
    meta = DeviceBuffer(ctx, 16 * n)
    ctx.h2d(sbuf.ptr, src, st)
    ctx.h2d(meta.ptr, np.concatenate([soff, doff]), st)
    engine.unshuffle_chunks(ctx, sbuf.ptr, meta.ptr, dbuf.ptr, meta.ptr + 8 * n, n, nbytes, es, st)
    out = np.zeros(dsize, dtype=np.uint8)
    ctx.d2h(out, dbuf.ptr, st)
    ctx.synchronize(st)
    for k, c in enumerate(chunks):
        want = np.frombuffer(memoryview(ref.unshuffle(c.tobytes(), es)), dtype=np.uint8)[:nbytes]
        got = out[doff[k]:doff[k] + nbytes]
        # numcodecs leaves the len % es tail untouched (zeros); HDF5 copies it
        # (SURVEY 8c): compare the shuffled body, and the tail as copied
        body = (nbytes // es) * es
        np.testing.assert_array_equal(got[:body], want[:body], err_msg=f"chunk {k}")
        np.testing.assert_array_equal(got[body:], c[body:], err_msg=f"chunk {k} tail")


def test_unshuffle_chunks_refuses_other_sizes(gpu):
    with pytest.raises(NotImplementedError):
        engine.unshuffle_chunks(gpu, 0, 0, 0, 0, 1, 64, 3, gpu.thread_stream())
