"""Minimal CBOR (RFC 8949) codec for the Reductionist wire format.

The reference client decodes Reductionist responses with ``cbor2.loads``
(``activestorage/reductionist.py:225``); ``cbor2`` is not part of this image,
so the subset the wire format needs is implemented here: unsigned and
negative integers (major types 0/1), byte and text strings (2/3, definite and
indefinite length), arrays (4), maps (5), tags (6, decoded as their content),
simple values false/true/null/undefined and half/single/double floats (7).
"""
from __future__ import annotations

import struct


class CBORError(ValueError):
    pass


def _head(major: int, n: int) -> bytes:
    if n < 24:
        return bytes([(major << 5) | n])
    if n < 1 << 8:
        return bytes([(major << 5) | 24, n])
    if n < 1 << 16:
        return bytes([(major << 5) | 25]) + struct.pack(">H", n)
    if n < 1 << 32:
        return bytes([(major << 5) | 26]) + struct.pack(">I", n)
    if n < 1 << 64:
        return bytes([(major << 5) | 27]) + struct.pack(">Q", n)
    raise CBORError("integer too large for CBOR")


def dumps(obj) -> bytes:
    """Encode ``obj`` (None, bool, int, float, str, bytes, list/tuple, dict)."""
    out = bytearray()
    _enc(obj, out)
    return bytes(out)


def _enc(obj, out: bytearray) -> None:
    import numpy as np
    if obj is None:
        out.append(0xF6)
    elif obj is True or obj is False:
        out.append(0xF5 if obj else 0xF4)
    elif isinstance(obj, (int, np.integer)):
        v = int(obj)
        out += _head(0, v) if v >= 0 else _head(1, -1 - v)
    elif isinstance(obj, (float, np.floating)):
        out += b"\xfb" + struct.pack(">d", float(obj))
    elif isinstance(obj, (bytes, bytearray, memoryview)):
        b = bytes(obj)
        out += _head(2, len(b)) + b
    elif isinstance(obj, str):
        b = obj.encode("utf-8")
        out += _head(3, len(b)) + b
    elif isinstance(obj, (list, tuple)):
        out += _head(4, len(obj))
        for x in obj:
            _enc(x, out)
    elif isinstance(obj, dict):
        out += _head(5, len(obj))
        for k, v in obj.items():
            _enc(k, out)
            _enc(v, out)
    else:
        raise CBORError(f"cannot encode {type(obj).__name__}")


def loads(data: bytes):
    """Decode one CBOR data item; trailing bytes are an error."""
    obj, pos = _dec(memoryview(bytes(data)), 0)
    if pos != len(data):
        raise CBORError("trailing bytes after CBOR item")
    return obj


_BREAK = object()


def _arg(buf, pos, info):
    if info < 24:
        return info, pos
    if info == 24:
        return buf[pos], pos + 1
    if info == 25:
        return struct.unpack_from(">H", buf, pos)[0], pos + 2
    if info == 26:
        return struct.unpack_from(">I", buf, pos)[0], pos + 4
    if info == 27:
        return struct.unpack_from(">Q", buf, pos)[0], pos + 8
    raise CBORError(f"reserved additional information {info}")


def _half(h: int) -> float:
    return struct.unpack(">e", struct.pack(">H", h))[0]


def _dec(buf, pos):
    if pos >= len(buf):
        raise CBORError("truncated CBOR")
    ib = buf[pos]
    pos += 1
    major, info = ib >> 5, ib & 31
    if major == 7:
        if info == 20:
            return False, pos
        if info == 21:
            return True, pos
        if info in (22, 23):
            return None, pos
        if info == 25:
            return _half(struct.unpack_from(">H", buf, pos)[0]), pos + 2
        if info == 26:
            return struct.unpack_from(">f", buf, pos)[0], pos + 4
        if info == 27:
            return struct.unpack_from(">d", buf, pos)[0], pos + 8
        if info == 31:
            return _BREAK, pos
        if info < 24:
            return info, pos
        if info == 24:
            return buf[pos], pos + 1
        raise CBORError(f"unsupported simple value {info}")
    if info == 31:   # indefinite length
        if major in (2, 3):
            parts = []
            while True:
                item, pos = _dec(buf, pos)
                if item is _BREAK:
                    break
                parts.append(item)
            return (b"".join(parts) if major == 2 else "".join(parts)), pos
        if major == 4:
            items = []
            while True:
                item, pos = _dec(buf, pos)
                if item is _BREAK:
                    return items, pos
                items.append(item)
        if major == 5:
            d = {}
            while True:
                k, pos = _dec(buf, pos)
                if k is _BREAK:
                    return d, pos
                v, pos = _dec(buf, pos)
                d[k] = v
        raise CBORError("indefinite length on a non-container")
    n, pos = _arg(buf, pos, info)
    if major == 0:
        return n, pos
    if major == 1:
        return -1 - n, pos
    if major in (2, 3):
        if pos + n > len(buf):
            raise CBORError("truncated CBOR string")
        b = bytes(buf[pos:pos + n])
        return (b if major == 2 else b.decode("utf-8")), pos + n
    if major == 4:
        items = []
        for _ in range(n):
            item, pos = _dec(buf, pos)
            items.append(item)
        return items, pos
    if major == 5:
        d = {}
        for _ in range(n):
            k, pos = _dec(buf, pos)
            v, pos = _dec(buf, pos)
            d[k] = v
        return d, pos
    # major 6: tag -> its content
    return _dec(buf, pos)
