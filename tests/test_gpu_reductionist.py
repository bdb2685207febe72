"""Row f4 on the GPU: the Reductionist-compatible server over real HTTP.

Requests are built the way the reference client builds them
(``activestorage/reductionist.py:176-217``: dtype name + byte_order, offset,
size, order, shape, selection as [start, stop, step], compression/filters
ids, one missing-data rule with f32 values widened to f64, axis), posted to
``/v2/{operation}/`` and decoded the way ``decode_result`` does
(``reductionist.py:222-239``).  Expected values: the CPU oracle
(``oracle/storage_ref.py``, the reference's storage.py algorithm) on the same
object bytes, with the missing tuple the request denotes.
"""
import sys
import zlib

import numpy as np
import pytest
import requests

from oracle import storage_ref as ref
from pyactivestorage_amd import reductionist_server as rs
from tests.test_reductionist_wire import client_decode

pytestmark = pytest.mark.gpu

SHAPE = (10, 12, 16)


@pytest.fixture(scope="module")
def server(tmp_path_factory, gpu):
    root = tmp_path_factory.mktemp("objects")
    (root / "bucket").mkdir()
    rng = np.random.default_rng(7)
    objs = {}
    blob = bytearray()

    def add(name, arr, shuffle=False, deflate=False):
        raw = arr.tobytes()
        if shuffle:
            raw = np.frombuffer(raw, np.uint8).reshape(-1, arr.itemsize).T.copy().tobytes()
        if deflate:
            raw = zlib.compress(raw, 4)
        objs[name] = (len(blob), len(raw), arr.dtype, shuffle, deflate)
        blob.extend(raw)

    f = rng.uniform(-50, 150, size=SHAPE).astype("<f4")
    f.reshape(-1)[::13] = 42.0
    add("f4", f)
    add("f8_shuf_zlib_be", rng.uniform(-5, 5, size=SHAPE).astype(">f8"), shuffle=True, deflate=True)
    i = rng.integers(-300, 300, size=SHAPE).astype("<i2")
    i.reshape(-1)[::7] = -7
    add("i2_shuf", i, shuffle=True)
    (root / "bucket" / "var.bin").write_bytes(bytes(blob))
    srv = rs.ReductionistServer(str(root), ("127.0.0.1", 0))
    srv.start()
    yield srv, str(root / "bucket" / "var.bin"), objs
    srv.shutdown()
    srv.server_close()


def build(url, offset, size, dtype, shape, sel, shuffle, deflate, missing, axis):
    """The reference client's request body (reductionist.py:176-217)."""
    body = {"interface_type": "s3", "url": url, "dtype": dtype.name,
            "byte_order": {"<": "little", ">": "big", "=": sys.byteorder, "|": sys.byteorder}[dtype.byteorder],
            "offset": int(offset), "size": int(size), "order": "C", "shape": list(shape)}
    if sel is not None:
        body["selection"] = [[s.start, s.stop, s.step] for s in sel]
    if deflate:
        body["compression"] = {"id": "zlib"}
    if shuffle:
        body["filters"] = [{"id": "shuffle", "element_size": dtype.itemsize}]
    if missing:
        body["missing"] = missing
    if axis is not None:
        body["axis"] = list(axis)
    return body


MISSING = [None, {"missing_value": 42.0}, {"missing_values": [42.0, -7.0]},
           {"valid_min": 0.0}, {"valid_max": 100.0}, {"valid_range": [-20.0, 90.0]}]
SELS = [None, (slice(1, 9, 2), slice(0, 12, 1), slice(3, 16, 4))]
AXES = [None, (0,), (1, 2)]


@pytest.mark.parametrize("name", ["f4", "f8_shuf_zlib_be", "i2_shuf"])
@pytest.mark.parametrize("op", ["sum", "min", "max", "count", "select"])
def test_server_matches_oracle(server, name, op):
    srv, path, objs = server
    off, size, dt, shuf, defl = objs[name]
    comp = ref.Zlib() if defl else None
    filt = [ref.Shuffle(dt.itemsize)] if shuf else None
    for miss in MISSING:
        m4 = rs.decode_missing(miss, dt)
        for sel in SELS:
            for axis in (AXES if op != "select" else [None]):
                body = build("s3://bucket/var.bin", off, size, dt, SHAPE, sel, shuf, defl, miss, axis)
                r = requests.post(f"{srv.url}/v2/{op}/", json=body, timeout=60)
                assert r.status_code == 200, r.text
                res, count = client_decode(r.content)
                s = sel or tuple(slice(0, n, 1) for n in SHAPE)
                ax = axis if axis is not None else (0, 1, 2)
                method = {"sum": np.ma.sum, "min": np.ma.min, "max": np.ma.max, "count": np.ma.sum,
                          "select": None}[op]
                want, wn = ref.reduce_chunk(path, off, size, comp, filt, m4, dt, SHAPE, "C", s, ax, method)
                if op == "select":
                    want_n = np.ma.count(want)
                    np.testing.assert_array_equal(np.asarray(res), np.ma.filled(want, 0))
                    assert count == want_n
                    continue
                wn = np.asarray(wn)
                np.testing.assert_array_equal(np.asarray(count), wn)
                if op == "count":
                    np.testing.assert_array_equal(np.asarray(res), wn)
                    continue
                w = np.ma.filled(want, 0)
                assert np.asarray(res).shape == w.shape
                if dt.kind == "f" and op == "sum":
                    np.testing.assert_allclose(np.asarray(res), w, rtol=1e-6, atol=1e-9)
                else:
                    np.testing.assert_array_equal(np.asarray(res), w)


def test_server_errors(server):
    srv, _, objs = server
    off, size, dt, _, _ = objs["f4"]
    body = build("s3://bucket/none.bin", off, size, dt, SHAPE, None, False, False, None, None)
    assert requests.post(f"{srv.url}/v2/sum/", json=body, timeout=30).status_code == 404
    body = build("s3://bucket/var.bin", off, size, dt, (7, 7), None, False, False, None, None)
    r = requests.post(f"{srv.url}/v2/sum/", json=body, timeout=30)
    assert r.status_code == 400 and "reshape" in r.json()["error"]["message"]
    assert requests.post(f"{srv.url}/v2/median/", json=body, timeout=30).status_code == 404
    assert requests.post(f"{srv.url}/v1/sum/", json=body, timeout=30).status_code == 404
