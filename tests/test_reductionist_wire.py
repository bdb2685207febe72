"""Row f4 host logic (no GPU): the CBOR codec and the Reductionist request /
response mapping.

Request payloads are the ones the reference client builds, as asserted in
the reference's own tests (``tests/unit/test_reductionist.py:70-78``,
``:125-150`` and the missing-data encodings at ``:157-199``), restated here
as data.  Responses are decoded exactly as ``decode_result`` does
(``activestorage/reductionist.py:222-239``: ``cbor.loads`` ->
``np.frombuffer(bytes, dtype).reshape(shape)`` -> mask where count == 0).
"""
import json
import sys

import numpy as np
import pytest

from pyactivestorage_amd import cbor
from pyactivestorage_amd import reductionist_server as rs


# RFC 8949 Appendix A examples (encoded hex -> value)
RFC_VECTORS = [
    ("00", 0), ("17", 23), ("1818", 24), ("1903e8", 1000), ("1a000f4240", 1000000),
    ("1b000000e8d4a51000", 1000000000000), ("20", -1), ("3863", -100), ("f4", False),
    ("f5", True), ("f6", None), ("fb3ff199999999999a", 1.1), ("f93c00", 1.0),
    ("fa47c35000", 100000.0), ("f97bff", 65504.0), ("40", b""), ("4401020304", b"\x01\x02\x03\x04"),
    ("60", ""), ("6161", "a"), ("6449455446", "IETF"), ("80", []), ("83010203", [1, 2, 3]),
    ("a0", {}), ("a201020304", {1: 2, 3: 4}), ("a26161016162820203", {"a": 1, "b": [2, 3]}),
    ("5f42010243030405ff", b"\x01\x02\x03\x04\x05"), ("9f018202039f0405ffff", [1, [2, 3], [4, 5]]),
    ("bf61610161629f0203ffff", {"a": 1, "b": [2, 3]}), ("c11a514b67b0", 1363896240),
]


@pytest.mark.parametrize("hexdata,value", RFC_VECTORS)
def test_cbor_rfc_vectors(hexdata, value):
    assert cbor.loads(bytes.fromhex(hexdata)) == value


@pytest.mark.parametrize("value", [0, 23, 24, 255, 256, 65535, 65536, 2**32, 2**63, -1, -24, -25,
                                   -2**63, 1.5, -0.0, "", "héllo", b"\x00" * 300, [1, [2, "x"]],
                                   {"bytes": b"ab", "dtype": "int32", "shape": [], "count": [2]}])
def test_cbor_roundtrip(value):
    assert cbor.loads(cbor.dumps(value)) == value


def test_cbor_errors():
    with pytest.raises(cbor.CBORError):
        cbor.loads(b"\x44\x01")          # truncated byte string
    with pytest.raises(cbor.CBORError):
        cbor.loads(b"\x01\x02")          # trailing bytes


def client_decode(payload):
    """reductionist.py:222-239 restated (the reference client's decoding)."""
    r = cbor.loads(payload)
    result = np.frombuffer(r["bytes"], dtype=r["dtype"])
    result = result.reshape(r["shape"] if "shape" in r else None)
    count = r["count"]
    return np.ma.masked_where(count == 0, result), count


def test_decode_request_defaults():
    """tests/unit/test_reductionist.py:70-78 payload."""
    body = {"interface_type": "s3", "url": "https://active.example.com", "dtype": "int32",
            "byte_order": sys.byteorder, "offset": 0, "size": 0}
    r = rs.decode_request("min", json.loads(json.dumps(body)))
    assert r["dtype"] == np.dtype("int32")
    assert r["offset"] == 0 and r["size"] == 0
    assert r["shape"] is None and r["selection"] is None and r["axis"] is None
    assert r["compression"] is None and r["filters"] is None
    assert r["missing"] == (None, None, None, None)


def test_decode_request_compression_filters():
    """tests/unit/test_reductionist.py:125-150 payload."""
    body = {"interface_type": "s3", "url": "https://active.example.com", "dtype": "int32",
            "byte_order": sys.byteorder, "offset": 2, "size": 128, "order": "C", "shape": [32],
            "selection": [[0, 2, 1]], "compression": {"id": "zlib"},
            "filters": [{"id": "shuffle", "element_size": 4}], "axis": [0]}
    r = rs.decode_request("min", json.loads(json.dumps(body)))
    assert r["shape"] == (32,) and r["selection"] == (slice(0, 2, 1),) and r["axis"] == (0,)
    assert r["compression"].codec_id == "zlib"
    assert [f.elementsize for f in r["filters"]] == [4]


@pytest.mark.parametrize("missing,expect", [
    ({"missing_value": 42.0}, (None, np.float32(42.0), None, None)),
    ({"missing_value": -42.0}, (None, np.float32(-42.0), None, None)),
    ({"valid_min": float(np.float32(-1e6))}, (None, None, np.float32(-1e6), None)),
    ({"valid_max": float(np.float32(1e6))}, (None, None, None, np.float32(1e6))),
    ({"valid_range": [float(np.float32(-1e6)), float(np.float32(1e6))]},
     (None, None, np.float32(-1e6), np.float32(1e6))),
])
def test_decode_missing(missing, expect):
    """Encodings of tests/unit/test_reductionist.py:157-199, values of the data type."""
    got = rs.decode_missing(missing, np.dtype("float32"))
    for g, e in zip(got, expect):
        assert (g is None and e is None) or (type(g) is type(e) and g == e)


def test_decode_missing_values_membership():
    """missing_values is membership (any listed value), carried by the two
    equality rules; duplicates collapse; more than two distinct values are
    refused."""
    got = rs.decode_missing({"missing_values": [42.0, -42.0]}, np.dtype(">f4"))
    assert got[2:] == (None, None)
    assert type(got[0]) is np.float32 and {float(got[0]), float(got[1])} == {42.0, -42.0}
    got = rs.decode_missing({"missing_values": [7, 7]}, np.dtype("<i2"))
    assert got == (None, np.int16(7), None, None)
    with pytest.raises(rs.RequestError):
        rs.decode_missing({"missing_values": [1.0, 2.0, 3.0]}, np.dtype("<f4"))


@pytest.mark.parametrize("body,status", [
    ({"dtype": "int32"}, 400),                                       # no url
    ({"url": "s3://b/k", "dtype": "complex64"}, 400),
    ({"url": "s3://b/k", "dtype": "int32", "byte_order": "middle"}, 400),
    ({"url": "s3://b/k", "dtype": "int32", "compression": {"id": "lz4"}}, 400),
    ({"url": "s3://b/k", "dtype": "int32", "filters": [{"id": "delta"}]}, 400),
    ({"url": "s3://b/k", "dtype": "int32", "missing": {"valid_range": [2, 1]}}, 400),
    ({"url": "s3://b/k", "dtype": "int32", "selection": [[0, 2, 0]]}, 400),
])
def test_decode_request_rejects(body, status):
    with pytest.raises(rs.RequestError) as e:
        rs.decode_request("sum", body)
    assert e.value.status == status


def test_unknown_operation_and_urls(tmp_path):
    with pytest.raises(rs.RequestError) as e:
        rs.decode_request("median", {"url": "s3://b/k", "dtype": "int32"})
    assert e.value.status == 404
    (tmp_path / "bucket").mkdir()
    (tmp_path / "bucket" / "obj").write_bytes(b"\x00" * 8)
    assert rs.resolve_url("s3://bucket/obj", str(tmp_path)).endswith("bucket/obj")
    assert rs.resolve_url("http://127.0.0.1:9000/bucket/obj", str(tmp_path)).endswith("bucket/obj")
    for url, st in (("s3://bucket/none", 404), ("s3://bucket/../../etc/passwd", 403), ("ftp://x/y", 400)):
        with pytest.raises(rs.RequestError) as e:
            rs.resolve_url(url, str(tmp_path))
        assert e.value.status == st
    status, ctype, payload = rs.handle("sum", b"{not json", str(tmp_path))
    assert status == 400 and ctype == "application/json" and b"invalid JSON" in payload


def test_encode_response_roundtrip():
    vals = np.array([[[1.5]]], dtype=">f4")
    cnt = np.array([[[7]]], dtype=np.int64)
    res, count = client_decode(rs.encode_response(vals, cnt))
    assert res.dtype == np.dtype("float32") and res.shape == (1, 1, 1) and res[0, 0, 0] == 1.5
    assert count == [[[7]]]
    res, count = client_decode(rs.encode_response(np.int64(12), np.int64(3)))
    assert res.size == 1 and int(np.asarray(res).reshape(-1)[0]) == 12 and count == 3


def test_execute_bounds_requests_before_any_allocation(tmp_path):
    """client-chosen offset/size/shape must not size pinned or
    device buffers beyond the object (400, before the GPU is touched)."""
    (tmp_path / "b").mkdir()
    (tmp_path / "b" / "o.bin").write_bytes(np.zeros(1024, "<f4").tobytes())
    base = {"url": "s3://b/o.bin", "dtype": "float32"}

    def run(**kw):
        body = dict(base, **kw)
        status, _, payload = rs.handle("sum", json.dumps(body).encode(), str(tmp_path))
        return status, payload

    for kw in ({"offset": 8192, "size": 4}, {"offset": 0, "size": 1 << 40}, {"offset": 4096, "size": 8},
               {"offset": 0, "size": 4096, "shape": [1 << 20, 1 << 20]}):
        status, payload = run(**kw)
        assert status == 400, (kw, status, payload)
        assert b"beyond" in payload or b"limit" in payload, payload
