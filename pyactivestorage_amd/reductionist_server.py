"""Reductionist-compatible wire front end (row f4) serving the GPU backend.

The reference's remote path (``interface_type="s3"``/``"https"``,
``activestorage/active.py:687-751``) posts one JSON request per chunk to a
Reductionist server at ``{server}/v2/{operation}/`` (``reductionist.py:92-99``),
built by ``build_request_data`` (``reductionist.py:176-217``), and decodes a
CBOR map ``{bytes, dtype, shape, count}`` (``decode_result``,
``reductionist.py:222-239``).  This module is such a server: it decodes the
request into the arguments of the drop-in ``reduce_chunk``
(:mod:`pyactivestorage_amd.storage`, i.e. the fused HIP kernel), runs it on the
GPU and encodes the answer, so the reference client works against it
unchanged.

Object URLs are served from a local directory (``root``): ``s3://bucket/key``
and ``http(s)://host[:port]/bucket/key`` both map to ``root/bucket/key``
(Reductionist's own object store access — S3, auth, caching — is out of
scope).

Semantics (a Reductionist request carries one masking rule, and its values
are of the data type, ``reductionist.py:147-173``):

* ``missing_value`` / ``missing_values`` mask by equality (``missing_values``:
  membership in the list, at most two distinct values), ``valid_min`` /
  ``valid_max`` / ``valid_range`` by range, each value first converted to the
  data type;
* reductions keep the reduced axes (``keepdims``), so ``Active`` can place
  the result at its ``out_selection`` exactly as with the local
  ``reduce_chunk`` (``active.py:778-799``); ``count`` has the result's shape;
* masked outputs (count 0) carry 0 in ``bytes``;
* ``mean`` answers sum / count (the reference client never sends it: it asks
  for ``sum``, ``reductionist.py:98``).
"""
from __future__ import annotations

import http.server
import json
import os
import sys
import threading
import urllib.parse
import zlib

import numpy as np

from . import cbor
from .storage import Shuffle, Zlib, reduce_chunk

OPERATIONS = ("count", "max", "mean", "min", "select", "sum")


class RequestError(Exception):
    """A request the server rejects; ``status`` is the HTTP status code."""

    def __init__(self, message, status=400):
        super().__init__(message)
        self.status = status


class GZip:
    """``compression: {"id": "gzip"}``: gzip-wrapped DEFLATE, inflated on the
    host (the device inflater reads zlib streams)."""

    codec_id = "gzip"

    def decode(self, buf, out=None):
        return zlib.decompress(bytes(buf), 31)


def _dtype(name, byte_order):
    try:
        dt = np.dtype(name)
    except TypeError as exc:
        raise RequestError(f"unsupported dtype {name!r}") from exc
    if dt.kind not in "iuf":
        raise RequestError(f"unsupported dtype {name!r}")
    if byte_order not in (None, "little", "big"):
        raise RequestError(f"invalid byte_order {byte_order!r}")
    if byte_order is not None and dt.itemsize > 1:
        dt = dt.newbyteorder("<" if byte_order == "little" else ">")
    return dt


def _value(v, dt):
    """A JSON number as a value of the data type (Reductionist's convention)."""
    if not isinstance(v, (int, float)) or isinstance(v, bool):
        raise RequestError(f"missing-data value {v!r} is not a number")
    return dt.newbyteorder("=").type(v)


def decode_missing(m, dt):
    """Reductionist ``missing`` object -> storage.py's 4-tuple
    ``(fill_value, missing_value, valid_min, valid_max)``."""
    if m is None:
        return (None, None, None, None)
    if not isinstance(m, dict) or len(m) != 1:
        raise RequestError("missing must be an object with exactly one key")
    (k, v), = m.items()
    if k == "missing_value":
        return (None, _value(v, dt), None, None)
    if k == "missing_values":
        # Reductionist masks elements equal to ANY listed value (membership),
        # unlike storage.py's broadcast ``==`` for array attributes
        # (storage.py:133-143).  Membership in up to two distinct values maps
        # onto the device mask's two equality rules (fill, missing).
        if not isinstance(v, list) or not v:
            raise RequestError("missing_values must be a non-empty list")
        vals = []
        for x in v:
            x = _value(x, dt)
            if not any(x == y for y in vals):
                vals.append(x)
        if len(vals) > 2:
            raise RequestError("at most 2 distinct missing_values are supported", 400)
        return (vals[1] if len(vals) == 2 else None, vals[0], None, None)
    if k == "valid_min":
        return (None, None, _value(v, dt), None)
    if k == "valid_max":
        return (None, None, None, _value(v, dt))
    if k == "valid_range":
        if not isinstance(v, list) or len(v) != 2:
            raise RequestError("valid_range must be [min, max]")
        lo, hi = _value(v[0], dt), _value(v[1], dt)
        if lo > hi:
            raise RequestError("valid_range min is greater than max")
        return (None, None, lo, hi)
    raise RequestError(f"unknown missing-data kind {k!r}")


def decode_request(operation: str, body: dict) -> dict:
    """JSON request (``reductionist.py:176-217``) -> ``reduce_chunk`` arguments."""
    if operation not in OPERATIONS:
        raise RequestError(f"unknown operation {operation!r}", 404)
    if not isinstance(body, dict):
        raise RequestError("request body must be a JSON object")
    for key in ("url", "dtype"):
        if key not in body:
            raise RequestError(f"missing field {key!r}")
    dt = _dtype(body["dtype"], body.get("byte_order"))
    offset, size = int(body.get("offset", 0)), body.get("size")
    if offset < 0 or (size is not None and int(size) < 0):
        raise RequestError("offset and size must be non-negative")
    shape = body.get("shape")
    if shape is not None:
        shape = tuple(int(s) for s in shape)
    order = body.get("order", "C")
    if order not in ("C", "F"):
        raise RequestError(f"invalid order {order!r}")
    sel = body.get("selection")
    if sel is not None:
        try:
            sel = tuple(slice(int(a), int(b), int(c)) for a, b, c in sel)
        except (TypeError, ValueError) as exc:
            raise RequestError("selection must be a list of [start, stop, step]") from exc
        if any(s.step == 0 for s in sel):
            raise RequestError("selection step must be non-zero")
    comp = body.get("compression")
    if comp is not None:
        cid = comp.get("id") if isinstance(comp, dict) else None
        if cid == "zlib":
            comp = Zlib()
        elif cid == "gzip":
            comp = GZip()
        else:
            raise RequestError(f"unsupported compression {comp!r}")
    filters = []
    for f in body.get("filters") or []:
        if not isinstance(f, dict) or f.get("id") != "shuffle":
            raise RequestError(f"unsupported filter {f!r}")
        filters.append(Shuffle(int(f.get("element_size", dt.itemsize))))
    axis = body.get("axis")
    if axis is not None:
        axis = tuple(int(a) for a in ([axis] if isinstance(axis, int) else axis))
    return {"url": body["url"], "offset": offset, "size": None if size is None else int(size),
            "compression": comp, "filters": filters or None,
            "missing": decode_missing(body.get("missing"), dt), "dtype": dt, "shape": shape,
            "order": order, "selection": sel, "axis": axis,
            "interface_type": body.get("interface_type", "s3")}


def resolve_url(url: str, root: str) -> str:
    """Object URL -> file under ``root`` (``s3://bucket/key`` or
    ``http(s)://host/bucket/key`` -> ``root/bucket/key``)."""
    p = urllib.parse.urlparse(url)
    if p.scheme == "s3":
        rel = p.netloc + "/" + p.path.lstrip("/")
    elif p.scheme in ("http", "https"):
        rel = p.path.lstrip("/")
    else:
        raise RequestError(f"unsupported URL scheme in {url!r}")
    rel = urllib.parse.unquote(rel)
    base = os.path.realpath(root)
    path = os.path.realpath(os.path.join(base, rel))
    if path != base and not path.startswith(base + os.sep):
        raise RequestError(f"object {url!r} is outside the served root", 403)
    if not os.path.isfile(path):
        raise RequestError(f"object {url!r} not found", 404)
    return path


_METHODS = {"sum": np.ma.sum, "min": np.ma.min, "max": np.ma.max, "mean": np.ma.sum,
            "count": np.ma.sum, "select": None}


# Largest decoded chunk a request may ask for (its shape x itemsize): the
# server sizes device and pinned buffers from it, so a client must not be
# able to request arbitrary allocations.
MAX_CHUNK_BYTES = int(os.environ.get("PYAS_SERVER_MAX_CHUNK_BYTES", str(1 << 30)))


def execute(operation: str, req: dict, root: str):
    """Run the request on the GPU; returns ``(values ndarray, count ndarray)``."""
    path = resolve_url(req["url"], root)
    dt = req["dtype"]
    size = req["size"]
    length = os.path.getsize(path)
    if req["offset"] > length:
        raise RequestError(f"offset {req['offset']} beyond the object's {length} bytes")
    if size is None or size == 0:   # Reductionist: 0/absent = to the end of the object
        size = length - req["offset"]
    if req["offset"] + size > length:
        raise RequestError(f"byte range [{req['offset']}, {req['offset'] + size}) beyond the "
                           f"object's {length} bytes")
    shape = req["shape"] or (size // dt.itemsize,)
    if int(np.prod(shape, dtype=np.float64)) * dt.itemsize > MAX_CHUNK_BYTES or \
            (req["compression"] is None and size > MAX_CHUNK_BYTES):
        raise RequestError(f"chunk larger than the server's {MAX_CHUNK_BYTES}-byte limit")
    sel = req["selection"]
    if sel is None:
        sel = tuple(slice(0, n, 1) for n in shape)
    axis = req["axis"] if req["axis"] is not None else tuple(range(len(shape)))
    tmp, n = reduce_chunk(path, req["offset"], size, req["compression"], req["filters"],
                          req["missing"], dt, shape, req["order"], sel, axis,
                          method=_METHODS[operation])
    if operation == "select":
        count = np.asarray(np.ma.count(tmp), dtype=np.int64)
        return np.ma.filled(tmp, 0), count
    n = np.asarray(n, dtype=np.int64)
    if operation == "count":
        return n, n
    vals = np.ma.filled(tmp, 0)
    if operation == "mean":
        with np.errstate(invalid="ignore", divide="ignore"):
            vals = np.where(n > 0, vals / np.maximum(n, 1), 0.0)
    return np.asarray(vals), n


def encode_response(values, count) -> bytes:
    """CBOR ``{bytes, dtype, shape, count}`` as ``decode_result`` reads it."""
    v = np.ascontiguousarray(values)
    if v.dtype.byteorder == ">" or (v.dtype.byteorder == "=" and sys.byteorder == "big"):
        v = v.astype(v.dtype.newbyteorder("<"))
    c = np.asarray(count, dtype=np.int64)
    return cbor.dumps({"bytes": v.tobytes(), "dtype": v.dtype.name, "shape": list(v.shape),
                       "count": c.tolist()})


def handle(operation: str, body: bytes, root: str):
    """One request -> ``(status, content_type, payload)``."""
    try:
        try:
            req = json.loads(body.decode("utf-8") if body else "null")
        except (UnicodeDecodeError, json.JSONDecodeError) as exc:
            raise RequestError(f"invalid JSON: {exc}") from exc
        vals, cnt = execute(operation, decode_request(operation, req), root)
        return 200, "application/cbor", encode_response(vals, cnt)
    except RequestError as exc:
        return exc.status, "application/json", _err(str(exc))
    except (ValueError, IndexError, TypeError, NotImplementedError, zlib.error) as exc:
        return 400, "application/json", _err(f"{type(exc).__name__}: {exc}")
    except FileNotFoundError as exc:
        return 404, "application/json", _err(str(exc))
    except Exception as exc:   # device / internal failure
        return 500, "application/json", _err(f"{type(exc).__name__}: {exc}")


def _err(msg):
    return json.dumps({"error": {"message": msg}}).encode()


class _Handler(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    # headers and body go out as two writes on a keep-alive connection:
    # without TCP_NODELAY, Nagle + the client's delayed ACK add ~40 ms each
    disable_nagle_algorithm = True

    def do_POST(self):  # noqa: N802 (http.server API)
        parts = [p for p in urllib.parse.urlparse(self.path).path.split("/") if p]
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n else b""
        if len(parts) != 2 or parts[0] != "v2":
            status, ctype, payload = 404, "application/json", _err(f"no route {self.path}")
        else:
            status, ctype, payload = handle(parts[1], body, self.server.root)
        self.send_response(status)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(payload)))
        self.end_headers()
        self.wfile.write(payload)

    def log_message(self, fmt, *args):  # quiet by default
        if self.server.verbose:
            super().log_message(fmt, *args)


class ReductionistServer(http.server.ThreadingHTTPServer):
    """``ReductionistServer(root, ("127.0.0.1", 0))``; ``.url`` is its base URL."""

    daemon_threads = True
    # the reference client opens one connection per pool thread at once
    # (active.py:557, up to max_threads): socketserver's default listen
    # backlog of 5 resets the rest
    request_queue_size = 256

    def __init__(self, root, address=("127.0.0.1", 8080), verbose=False, reuse_port=False):
        self.root = root
        self.verbose = verbose
        self.reuse_port = reuse_port
        super().__init__(address, _Handler)

    def server_bind(self):
        if self.reuse_port:   # worker processes share one port (the kernel balances)
            import socket
            self.socket.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
        super().server_bind()

    @property
    def url(self):
        host, port = self.server_address[:2]
        return f"http://{host}:{port}"

    def start(self):
        """Serve on a background thread; returns the thread."""
        t = threading.Thread(target=self.serve_forever, daemon=True)
        t.start()
        return t


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Reductionist-compatible server on the MI355X backend")
    ap.add_argument("root", help="directory holding the objects (bucket/key)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--workers", type=int, default=1,
                    help="server processes sharing the port (SO_REUSEPORT); each has its own "
                         "GPU context, so request handling scales past one Python interpreter")
    ap.add_argument("--reuse-port", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.workers > 1 and a.port == 0:
        ap.error("--workers needs a fixed --port")
    children = []
    if a.workers > 1:
        import signal
        import subprocess
        # SIGTERM ends serve_forever through the finally below, which stops the workers
        signal.signal(signal.SIGTERM, lambda *_: sys.exit(0))
        cmd = [sys.executable, "-m", "pyactivestorage_amd.reductionist_server", a.root,
               "--host", a.host, "--port", str(a.port), "--reuse-port"] + (["-v"] if a.verbose else [])
        # started before this process touches the GPU; children, not forks
        children = [subprocess.Popen(cmd) for _ in range(a.workers - 1)]
    srv = ReductionistServer(a.root, (a.host, a.port), a.verbose, reuse_port=a.reuse_port or a.workers > 1)
    if not a.reuse_port:
        print(f"serving {a.root} at {srv.url}/v2/<operation>/ ({a.workers} process(es))", flush=True)
    try:
        srv.serve_forever()
    finally:
        for ch in children:
            ch.terminate()
        for ch in children:
            ch.wait()


if __name__ == "__main__":
    main()
