"""GPU zlib inflate (row f3) against zlib itself and the reference's HDF5 files.

The reference decodes compressed chunks with numcodecs.Zlib -> zlib.decompress
(activestorage/hdf2numcodec.py:34-35, storage.py:119-120).  Parity is bit-exact:

* every gzip chunk of the reference's test files (tests/golden/h5_chunks.npz,
  extracted by extract_h5.py) inflates to the bytes whose SHA-256 libhdf5
  recorded (after HDF5's un-shuffle where the pipeline has one);
* streams made by this image's zlib across levels, strategies, window sizes,
  memory levels, data kinds and sizes (stored, fixed and dynamic blocks, codes
  longer than the 10-bit table, d=1 runs, 32 KiB distances) equal
  zlib.decompress;
* malformed streams raise zlib.error exactly where zlib.decompress does.
"""
import hashlib
import zlib

import numpy as np
import pytest

from oracle import storage_ref as ref
from pyactivestorage_amd.inflate import inflate_many
from tests import _golden as G

pytestmark = pytest.mark.gpu


def _field(n, seed=0):
    rng = np.random.default_rng(seed)
    x = np.cumsum(rng.normal(size=n)).astype(np.float32) + 280.0
    return x


def _shuffled(a):
    b = np.frombuffer(a.tobytes(), dtype=np.uint8).reshape(-1, a.dtype.itemsize)
    return b.T.copy().tobytes()


def _cases():
    rng = np.random.default_rng(1)
    field = _field(64 ** 3 // 4)
    text = b"".join(b"chunk %d of variable tas, value %.3f; " % (i, v) for i, v in enumerate(field[:4000]))
    payloads = {
        "zeros": bytes(1 << 20),
        "random": rng.integers(0, 256, 100_000, dtype=np.uint8).tobytes(),
        "field": field.tobytes(),
        "field_shuffled": _shuffled(field),
        "text": text,
        "one": b"x",
        "empty": b"",
        "k1023": rng.integers(0, 4, 1023, dtype=np.uint8).tobytes(),
        "k1025": rng.integers(0, 4, 1025, dtype=np.uint8).tobytes(),
        "far": rng.integers(0, 256, 40_000, dtype=np.uint8).tobytes() * 2,   # beyond the 32 KiB window
        "d12k": rng.integers(0, 256, 12_000, dtype=np.uint8).tobytes() * 3,   # matches past an 8 KiB ring
        "d20k": rng.integers(0, 256, 20_000, dtype=np.uint8).tobytes() * 3,   # ... and past 16 KiB
        "d32k": rng.integers(0, 256, 32_768, dtype=np.uint8).tobytes() * 2,   # the maximum distance
    }
    out = []
    for name, p in payloads.items():
        for level in (0, 1, 6, 9):
            out.append((f"{name}-l{level}", p, zlib.compress(p, level)))
    strategies = {"filtered": zlib.Z_FILTERED, "huffman": zlib.Z_HUFFMAN_ONLY, "rle": zlib.Z_RLE,
                  "fixed": zlib.Z_FIXED}
    for sname, st in strategies.items():
        for name in ("field_shuffled", "text", "zeros"):
            co = zlib.compressobj(6, zlib.DEFLATED, 15, 8, st)
            out.append((f"{name}-{sname}", payloads[name], co.compress(payloads[name]) + co.flush()))
    for wbits in (9, 12, 15):
        for mem in (1, 9):
            co = zlib.compressobj(9, zlib.DEFLATED, wbits, mem)
            p = payloads["text"]
            out.append((f"text-w{wbits}-m{mem}", p, co.compress(p) + co.flush()))
    # full-flush / sync-flush points put empty stored blocks mid-stream
    co = zlib.compressobj(6)
    p = payloads["field_shuffled"]
    s = co.compress(p[:100_000]) + co.flush(zlib.Z_SYNC_FLUSH) + co.compress(p[100_000:]) + co.flush()
    out.append(("sync-flush", p, s))
    return out


CASES = _cases()


def test_inflate_matches_zlib_all_cases(gpu):
    got = inflate_many(gpu, [c[2] for c in CASES], [max(len(c[1]), 1) for c in CASES])
    for (name, plain, comp), g in zip(CASES, got):
        assert zlib.decompress(comp) == plain, name
        assert g == plain, name


@pytest.mark.parametrize("wbits", [13, 14, 15])
def test_inflate_every_ring_size(gpu, wbits):
    """The LDS ring size is a per-context launch choice; each variant is exact."""
    sel = [c for c in CASES if c[0].startswith(("d12k", "d20k", "d32k", "text", "field_shuffled"))]
    fn = gpu.lib.pyas_ctx_set_inflate_window_bits
    assert fn(gpu.handle, wbits) == 0
    try:
        got = inflate_many(gpu, [c[2] for c in sel], [max(len(c[1]), 1) for c in sel])
    finally:
        fn(gpu.handle, 13)
    for (name, plain, _), g in zip(sel, got):
        assert g == plain, (name, wbits)


def test_inflate_trailing_bytes_ignored(gpu):
    p = _field(5000).tobytes()
    comp = zlib.compress(p, 6) + b"garbage after the adler trailer"
    assert zlib.decompress(comp) == p
    assert inflate_many(gpu, [comp], len(p)) == [p]


def test_inflate_reference_hdf5_chunks(gpu):
    """Every deflated chunk of the reference's test files (libhdf5-written)."""
    metas, blobs = G.h5_meta(), G.h5_blobs()
    n_checked = 0
    for key, meta in metas.items():
        ids = [f["id"] for f in meta["filters"]]
        if 1 not in ids:
            continue
        es = np.dtype(meta["dtype"]).itemsize
        nbytes = int(np.prod(meta["chunks"])) * es
        streams = [blobs[key][ch["blob_start"]: ch["blob_start"] + ch["size"]].tobytes()
                   for ch in meta["chunk_table"]]
        got = inflate_many(gpu, streams, nbytes)
        for ch, s, g in zip(meta["chunk_table"], streams, got):
            assert g == zlib.decompress(s), key
            dec = ref.unshuffle(g, es).tobytes() if 2 in ids else g
            assert hashlib.sha256(dec).hexdigest() == ch["hdf5_decoded_sha256"], (key, ch["coords"])
            n_checked += 1
    assert n_checked >= 18


def test_inflate_many_streams_unaligned(gpu):
    """Hundreds of streams, odd sizes and offsets (exercises unaligned src/dst)."""
    rng = np.random.default_rng(7)
    plains = [_shuffled(_field(int(n), seed=i)) for i, n in enumerate(rng.integers(1, 20_000, 300))]
    comps = [zlib.compress(p, int(lvl)) for p, lvl in zip(plains, rng.integers(0, 10, 300))]
    for sa, da in ((1, 1), (3, 16), (16, 256)):
        got = inflate_many(gpu, comps, [len(p) for p in plains], src_align=sa, dst_align=da)
        assert got == plains, (sa, da)


def _bits(*fields):
    """Pack (value, nbits) LSB-first; Huffman codes are given pre-reversed."""
    acc, n, out = 0, 0, bytearray()
    for v, k in fields:
        acc |= v << n
        n += k
    while n > 0:
        out.append(acc & 255)
        acc >>= 8
        n -= 8
    return bytes(out)


def _rev(code, n):
    return int(format(code, f"0{n}b")[::-1], 2)


def _bad_streams():
    good = zlib.compress(_field(3000).tobytes(), 6)
    zd = zlib.compressobj(6, zdict=b"preset dictionary")
    with_dict = zd.compress(b"abc") + zd.flush()
    hdr = b"\x78\x9c"
    far = hdr + _bits((1, 1), (1, 2), (_rev(0b0000001, 7), 7), (0, 5), (0, 7))   # match d=1 at pos 0
    stored_bad = hdr + bytes([0x01]) + (5).to_bytes(2, "little") + (5).to_bytes(2, "little") + b"abcde"
    return {
        "header": b"\x78\x9d" + good[2:],
        "method": b"\x79\x9c" + good[2:],
        "dict": with_dict,
        "block_type": hdr + bytes([0x07]) + bytes(8),
        "stored_len": stored_bad,
        "distance": far,
        "truncated": good[: len(good) // 2],
        "truncated_trailer": good[:-2],
        "checksum": good[:-1] + bytes([good[-1] ^ 1]),
        "short": b"\x78",
    }


@pytest.mark.parametrize("name", sorted(_bad_streams()))
def test_inflate_errors_match_zlib(gpu, name):
    s = _bad_streams()[name]
    with pytest.raises(zlib.error):
        zlib.decompress(s)
    with pytest.raises(zlib.error):
        inflate_many(gpu, [s], 1 << 16)


def test_inflate_overflow_is_value_error(gpu):
    p = bytes(5000)
    with pytest.raises(ValueError):
        inflate_many(gpu, [zlib.compress(p)], 4096)
