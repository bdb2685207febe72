"""Pin the CPU oracle against the reference itself (CPU-only tests).

* every golden case (tests/golden/reference_cases.json, produced by running
  the reference's own storage.py) is reproduced bit-exactly by the oracle,
  including the reference's exceptions;
* the oracle's restated un-shuffle equals libhdf5's shuffle decode on every
  netCDF numeric type and both byte orders, and its zlib+unshuffle decode of
  every chunk of the reference's test files hashes to libhdf5's decode;
* the reference's hard-coded unit-test answers (tests/unit/test_storage.py).
"""
import hashlib

import numpy as np
import pytest

from oracle import storage_ref as ref
from tests import _golden as G


@pytest.mark.parametrize("block", range(0, len(G.cases()), 200))
def test_oracle_reproduces_reference_outputs(block):
    cases = G.cases()
    for i in range(block, min(block + 200, len(cases))):
        a = G.args_of(i, ref.Zlib, ref.Shuffle)
        exp = G.expected(i)
        if isinstance(exp[0], str):
            with pytest.raises(Exception) as ei:
                ref.reduce_chunk_bytes(a["raw"], a["compression"], a["filters"], a["missing"], a["dtype"],
                                       a["shape"], a["order"], a["chunk_selection"], a["axis"], a["method"])
            assert type(ei.value).__name__ == exp[0], i
            continue
        tmp, n = ref.reduce_chunk_bytes(a["raw"], a["compression"], a["filters"], a["missing"], a["dtype"],
                                        a["shape"], a["order"], a["chunk_selection"], a["axis"], a["method"])
        G.check(i, tmp, n, rel=0)


def test_unshuffle_matches_libhdf5():
    z = np.load(G.os.path.join(G.HERE, "h5_shuffle.npz"))
    names = sorted({k.split(":")[0] for k in z.files})
    assert len(names) == 20
    for name in names:
        data = z[name + ":data"]
        raw = z[name + ":raw"].tobytes()
        got = ref.unshuffle(raw, data.dtype.itemsize)
        assert got.tobytes() == data.tobytes(), name


def test_decode_matches_libhdf5_hashes():
    meta, blobs = G.h5_meta(), G.h5_blobs()
    n = 0
    for key, v in meta.items():
        comp = ref.Zlib() if any(f["id"] == 1 for f in v["filters"]) else None
        filt = [ref.Shuffle(np.dtype(v["dtype"]).itemsize)] if any(f["id"] == 2 for f in v["filters"]) else None
        blob = blobs[key]
        for ch in v["chunk_table"]:
            raw = blob[ch["blob_start"]: ch["blob_start"] + ch["size"]].tobytes()
            dec = ref.decode_chunk(raw, comp, filt, v["dtype"], v["chunks"], "C")
            assert hashlib.sha256(np.ascontiguousarray(dec).tobytes()).hexdigest() == ch["hdf5_decoded_sha256"], key
            n += 1
    assert n >= 30


def test_reference_unit_answers():
    """tests/unit/test_storage.py known answers, through the oracle."""
    blobs = G.h5_blobs()
    tmp, n = ref.reduce_chunk_bytes(blobs["raw:cesm2_native.nc:2:128"].tobytes(), None, None,
                                    [None, 2050, None, None], "i2", (8, 8), "C", slice(0, 2, 1), (0, 1), np.min)
    assert tmp == -1 and n == 15                                   # test_storage.py:89-90
    full = (slice(0, 62, 1), slice(0, 2, 1), slice(0, 3, 1), slice(0, 2, 1))
    r, c = ref.reduce_chunk_bytes(blobs["raw:daily_data_masked.nc:6911:2976"].tobytes(), None, None,
                                  (None, 999.0, None, None), "float32", (62, 2, 3, 2), "C", full,
                                  (0, 1, 2, 3), np.mean)
    assert r == np.array([[[[249.45955882352942]]]]) and c == 680  # test_storage.py:118-119
    for miss in ((None, 999.0, None, None), (999., None, None, None), (None, None, 1000., None),
                 (None, None, None, 1.)):
        r, c = ref.reduce_chunk_bytes(blobs["raw:daily_data_fullmask.nc:6911:2976"].tobytes(), None, None,
                                      miss, "float32", (62, 2, 3, 2), "C", full, (0, 1, 2, 3), np.mean)
        assert r.size == 1 and c == 0                              # test_storage.py:143-144
    r, c = ref.reduce_chunk_bytes(blobs["raw:zero_chunked.nc:8760:48"].tobytes(), None, None,
                                  (None, None, None, None), "float32", (3, 4), "C",
                                  (slice(0, 3, 1), slice(0, 4, 1)), (0, 1), np.mean)
    assert r.size == 1 and r == 0 and c == 12                      # test_storage.py:243-245


def test_mask_missing_broadcast_semantics():
    """tests/unit/test_storage.py:9-67 on the oracle's mask_missing."""
    d1 = np.ma.array([[[-900., 33.], [33., -900], [33., 44.]]], mask=False, dtype=float)
    r1 = ref.mask_missing(d1, ([-900.], np.array([-900.]), None, None))
    assert np.array_equal(np.ma.getmaskarray(r1), [[[True, False], [False, True], [False, False]]])
    r2 = ref.mask_missing(d1, ([-900., 33.], np.array([-900., 33.]), None, None))
    assert np.array_equal(np.ma.getmaskarray(r2), [[[True, True], [False, False], [False, False]]])
    with pytest.raises(ValueError, match="not brodcastable"):
        ref.mask_missing(d1, (-900, np.array([-900., -900., 33.]), None, None))
