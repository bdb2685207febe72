"""Native file ingest sweep (row f2): page-cache-hot chunk-major file of the
C3 variable (4 GiB) -> pyas_read_ranges -> device, for several reader-thread
counts and staging-ring shapes.  Prints one JSON line per setting (GB/s)."""
import itertools
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pyactivestorage_amd.device import get_context
    from pyactivestorage_amd.ingest import read_ranges, set_slots
    ctx = get_context(0)
    nbytes, cb = 4 << 30, 1 << 20
    n = nbytes // cb
    path = os.path.join(tempfile.gettempdir(), f"pyas_ingest_{os.getpid()}.bin")
    try:
        blk = np.random.default_rng(0).integers(0, 255, size=256 << 20, dtype=np.uint8).tobytes()
        with open(path, "wb") as f:
            for _ in range(nbytes // len(blk)):
                f.write(blk)
        dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        offs = np.arange(n, dtype=np.int64) * cb
        sizes = np.full(n, cb, dtype=np.int64)
        for threads, (slots, mib) in itertools.product(
                (8, 16), ((8, 64), (4, 128), (16, 32), (16, 64), (8, 128), (32, 32))):
            set_slots(ctx, slots, mib << 20)
            read_ranges(ctx, path, offs, sizes, dev.data_ptr(), offs, st, threads)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                read_ranges(ctx, path, offs, sizes, dev.data_ptr(), offs, st, threads)
            torch.cuda.synchronize()
            sec = (time.perf_counter() - t0) / 3
            print(json.dumps({"threads": threads, "slots": slots, "slot_MiB": mib,
                              "GBps": round(nbytes / sec / 1e9, 2)}), flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
