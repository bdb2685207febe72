"""First-call cost of libpyas_hip.so: in a fresh process,
the time to dlopen the library, to create the first context (HIP runtime
start and code-object registration), and to run the first and a second
small reduction (the first includes loading the kernel's code object).

    python tools/lib_load_time.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    t0 = time.perf_counter()
    from pyactivestorage_amd import _lib
    lib = _lib.load()
    t1 = time.perf_counter()
    from pyactivestorage_amd.device import get_context
    ctx = get_context(0)
    t2 = time.perf_counter()
    from pyactivestorage_amd import storage
    raw = np.arange(16 * 16 * 16, dtype=np.float32).tobytes()
    none = (None, None, None, None)

    def one():
        return storage.reduce_chunk_bytes(raw, None, None, none, "<f4", (16, 16, 16), "C",
                                          (slice(None),) * 3, (0, 1, 2), np.ma.sum)
    one()
    t3 = time.perf_counter()
    one()
    t4 = time.perf_counter()
    path = _lib.LIB_PATH
    print(json.dumps({"lib": os.path.relpath(path, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      "lib_bytes": os.path.getsize(path),
                      "dlopen_ms": round((t1 - t0) * 1e3, 1),
                      "first_context_ms": round((t2 - t1) * 1e3, 1),
                      "first_reduce_ms": round((t3 - t2) * 1e3, 1),
                      "second_reduce_ms": round((t4 - t3) * 1e3, 2),
                      "abi": int(lib.pyas_abi_version())}))


if __name__ == "__main__":
    main()
