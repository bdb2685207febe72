"""ctypes binding of the C ABI in ``include/pyas.h`` (``lib/libpyas_hip.so``).

This is the only place Python touches the native library.  The product path
has no CPU fallback: if the shared library is missing or the HIP runtime has
no device, calls raise ``RuntimeError`` instead of silently computing on the
host.
"""
from __future__ import annotations

import ctypes
import os
import threading

MAX_DIMS = 8
ABI_VERSION = 2

# pyas_status
OK, EINVAL, ENOTSUP, EDEVICE, ENOMEM, EINDEX, EIO = range(7)
# pyas_dtype
I8, U8, I16, U16, I32, U32, I64, U64, F32, F64 = range(10)
# mask flags
MASK_EQ0, MASK_EQ1, MASK_GT, MASK_LT, MASK_TAB0, MASK_TAB1 = 1, 2, 4, 8, 16, 32
COMBINE_ROUND_TO_VAR = 1
# pyas_format_partials methods
FORMAT_SUM, FORMAT_MIN, FORMAT_MAX, FORMAT_MEAN = range(4)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# PYAS_LIB selects an alternative build (tuning experiments only)
LIB_PATH = os.environ.get("PYAS_LIB") or os.path.join(LIB_DIR, "libpyas_hip.so")


class Scalar(ctypes.Union):
    _fields_ = [("f", ctypes.c_double), ("i", ctypes.c_int64), ("u", ctypes.c_uint64)]


class Partial(ctypes.Structure):
    _fields_ = [("sum", Scalar), ("count", ctypes.c_int64), ("min", Scalar), ("max", Scalar)]


class Mask(ctypes.Structure):
    _fields_ = [
        ("flags", ctypes.c_uint32),
        ("tab_len", ctypes.c_int32 * 2),
        ("eq_lo", Scalar * 2),
        ("eq_hi", Scalar * 2),
        ("gt", Scalar),
        ("lt", Scalar),
        ("tab_lo", ctypes.c_void_p * 2),
        ("tab_hi", ctypes.c_void_p * 2),
        ("tab_stride", (ctypes.c_int64 * MAX_DIMS) * 2),
    ]


class Batch(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int32),
        ("byteswap", ctypes.c_int32),
        ("shuffle", ctypes.c_int32),
        ("ndim", ctypes.c_int32),
        ("chunk_shape", ctypes.c_int64 * MAX_DIMS),
        ("n_chunks", ctypes.c_int64),
        ("data", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("sel", ctypes.c_void_p),
        ("index_pool", ctypes.c_void_p),
    ]


class Grid(ctypes.Structure):
    """pyas_grid: per-dim tables of a box query for pyas_combine_grid."""
    _fields_ = [
        ("ndim", ctypes.c_int32),
        ("axes_mask", ctypes.c_uint32),
        ("n_coords", ctypes.c_int64 * MAX_DIMS),
        ("out_extent", ctypes.c_int64 * MAX_DIMS),
        ("pos_coord", ctypes.c_void_p * MAX_DIMS),
        ("pos_local", ctypes.c_void_p * MAX_DIMS),
        ("coord_count", ctypes.c_void_p * MAX_DIMS),
        ("chunk_out_offsets", ctypes.c_void_p),
    ]


class Scatter(ctypes.Structure):
    """pyas_scatter: output placement tables of pyas_select_scatter."""
    _fields_ = [
        ("pos", ctypes.c_void_p),
        ("chunk_base", ctypes.c_void_p),
        ("out_stride", ctypes.c_int64 * MAX_DIMS),
    ]


class TieGeom(ctypes.Structure):
    """pyas_tie_geom: how NumPy walks chunk[sel] (zerosign.geometry)."""
    _fields_ = [
        ("perm", ctypes.c_int32 * MAX_DIMS),
        ("flags", ctypes.c_uint32),
    ]


class ChunkDesc(ctypes.Structure):
    """pyas_chunk_desc: one chunk's layout for pyas_coalesced_reduce."""
    _fields_ = [
        ("dtype", ctypes.c_int32),
        ("byteswap", ctypes.c_int32),
        ("shuffle", ctypes.c_int32),
        ("ndim", ctypes.c_int32),
        ("chunk_shape", ctypes.c_int64 * MAX_DIMS),
        ("zlib", ctypes.c_int32),
        ("axes_mask", ctypes.c_uint32),
        ("tie_which", ctypes.c_uint32),
        ("tie", TieGeom),
    ]


class TieRule(ctypes.Structure):
    """pyas_tie_rule: NumPy's zero-sign tie rule (zerosign.py)."""
    _fields_ = [
        ("lanes", ctypes.c_int32),
        ("piece", ctypes.c_int32),
        ("acc", ctypes.c_int32),
        ("rank", ctypes.c_uint8 * 64),
        ("acc_rank", ctypes.c_uint8 * 64),
    ]


# compact per-output records of pyas_reduce_axes_ex (pyas.h PYAS_REC_*)
REC_FULL, REC_SUM, REC_MIN, REC_MAX = 0, 1, 2, 3
REC_ZERO_SIGN = 0x100    # pyas.h PYAS_REC_ZERO_SIGN: the per-chunk walk keys NumPy's zero sign
REC_DENSE_ONLY = 0x200   # pyas.h PYAS_REC_DENSE_ONLY: every chunk is dense-owned, no generic launch
REC_GENERIC_ONLY = 0x400  # pyas.h PYAS_REC_GENERIC_ONLY: no chunk is dense-owned, no dense launch
TIE_REC = 4


def rec_nbytes(itemsize: int, rec: int) -> int:
    """Bytes per output of a partial array of form ``rec``."""
    return 32 if rec == REC_FULL else (8 if itemsize <= 4 else 16)


def combine_rec(rec: int) -> int:
    """PYAS_COMBINE_REC(rec): combine flag of record inputs."""
    return int(rec) << 4


PARTIAL_NBYTES = ctypes.sizeof(Partial)
assert PARTIAL_NBYTES == 32

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_sz = ctypes.c_size_t

# name -> argtypes (restype is always c_int except the two noted)
SIGNATURES = {
    "pyas_abi_version": [],
    "pyas_last_error": [],
    "pyas_device_count": [ctypes.POINTER(ctypes.c_int)],
    "pyas_ctx_create": [ctypes.c_int, ctypes.POINTER(_vp)],
    "pyas_ctx_destroy": [_vp],
    "pyas_ctx_set_tile_bytes": [_vp, _i64],
    "pyas_ctx_set_inflate_window_bits": [_vp, _i32],
    "pyas_ctx_set_chained_combine": [_vp, _i32],
    "pyas_ctx_set_fold_min_blocks": [_vp, _i64],
    "pyas_ctx_set_tie_rule": [_vp, _i32, ctypes.POINTER(TieRule)],
    "pyas_tie_chunks": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), ctypes.POINTER(TieGeom), _u32, _u32,
                        _vp, _vp, _vp],
    "pyas_tie_chunks_total": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), ctypes.POINTER(TieGeom), _u32,
                              _vp, _i64, _i64, _vp],
    "pyas_tie_chunk_flags": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), ctypes.POINTER(TieGeom), _u32,
                             _u32, _vp, _vp, _i64, _vp, _vp],
    "pyas_tie_grid": [_vp, _i32, ctypes.POINTER(Grid), _vp, _vp, _i64, _u32, _vp, _vp, _vp],
    "pyas_tie_segments": [_vp, _i32, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _u32, _vp, _vp, _vp],
    "pyas_tie_keys_reset": [_vp, _vp, _i64, _vp],
    "pyas_tie_finalize": [_vp, _i32, _vp, _i64, _i32, _i64, _u32, _vp, _vp],
    "pyas_malloc": [_vp, _sz, ctypes.POINTER(_vp)],
    "pyas_free": [_vp, _vp],
    "pyas_host_alloc": [_vp, _sz, ctypes.POINTER(_vp)],
    "pyas_host_free": [_vp, _vp],
    "pyas_memcpy_h2d": [_vp, _vp, _vp, _sz, _vp],
    "pyas_memcpy_d2h": [_vp, _vp, _vp, _sz, _vp],
    "pyas_stream_create": [_vp, ctypes.POINTER(_vp)],
    "pyas_stream_destroy": [_vp, _vp],
    "pyas_stream_synchronize": [_vp, _vp],
    "pyas_stream_wait": [_vp, _vp, _vp],
    "pyas_reduce_chunks": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), _vp, _vp, _u32, _vp],
    "pyas_reduce_axes": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), _u32, _vp, _vp, _vp],
    "pyas_reduce_axes_ex": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), _u32, _i32, _vp, _vp, _vp],
    "pyas_select_chunks": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), _vp, _vp, _vp, _vp],
    "pyas_select_scatter": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), ctypes.POINTER(Scatter),
                            _vp, _vp, _vp],
    "pyas_combine_partials": [_vp, _i32, _vp, _i64, _u32, _vp, _vp],
    "pyas_reduce_sharded": [_vp, _vp, _vp, _i32, _u32, _vp, _vp],
    "pyas_reduce_sharded_tie": [_vp, _vp, _vp, _i32, _u32, _vp, _u32, _vp, _vp],
    "pyas_shard_release": [],
    "pyas_combine_segments": [_vp, _i32, _vp, _vp, _vp, _i64, _u32, _vp, _vp],
    "pyas_combine_grid": [_vp, _i32, _vp, ctypes.POINTER(Grid), _u32, _vp, _vp],
    "pyas_reduce_axes_grid": [_vp, ctypes.POINTER(Batch), ctypes.POINTER(Mask), ctypes.POINTER(Grid), _u32,
                              _vp, _vp],
    "pyas_format_partials": [_vp, _i32, _vp, _i64, _i32, _vp, _vp, _vp, _vp],
    "pyas_unshuffle": [_vp, _vp, _vp, _i64, _i32, _vp],
    "pyas_unshuffle_chunks": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pyas_inflate": [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "pyas_read_ranges": [_vp, ctypes.c_int, _i64, _vp, _vp, _vp, _vp, _i32, _vp],
    "pyas_read_ranges_zlib": [_vp, ctypes.c_int, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _i32, _vp],
    "pyas_ctx_set_ingest_slots": [_vp, _i32, _i64],
    "pyas_coalescer_create": [_vp, _i64, _i32, ctypes.POINTER(_vp)],
    "pyas_coalescer_destroy": [_vp],
    "pyas_coalescer_stats": [_vp, _vp],
    "pyas_coalesced_reduce": [_vp, ctypes.c_char_p, _i64, _i64, ctypes.POINTER(ChunkDesc), ctypes.POINTER(Mask),
                              _vp, _vp, _i32, _i64, _vp, _vp],
    "pyas_timing_enable": [_vp, _i32],
    "pyas_timing_read": [_vp, ctypes.POINTER(ctypes.c_float), _i32, ctypes.POINTER(_i32)],
}

_lock = threading.Lock()
_lib = None


def load(path: str | None = None):
    """Load (once) and return the ctypes library handle.

    Raises ``RuntimeError`` if the library has not been built: there is no
    host fallback for the reduction path.
    """
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"pyactivestorage_amd: HIP library not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C "
                "pyactivestorage_amd/csrc). There is no CPU fallback.")
        lib = ctypes.CDLL(p)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_char_p if name == "pyas_last_error" else ctypes.c_int
        if lib.pyas_abi_version() != ABI_VERSION:
            raise RuntimeError("pyactivestorage_amd: ABI version mismatch with " + p + " (rebuild it)")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    """Map a pyas_status to the exception type the reference raises."""
    if rc == OK:
        return
    msg = (load().pyas_last_error() or b"").decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == EINVAL:
        raise ValueError(text)
    if rc == ENOTSUP:
        raise NotImplementedError(text)
    if rc == EINDEX:
        raise IndexError(text)
    if rc == ENOMEM:
        raise MemoryError(text)
    if rc == EIO:
        raise OSError(text)
    raise RuntimeError(text)
