"""cProfile of single-thread per-chunk reduce_chunk calls (host costs)."""
import cProfile
import os
import pstats
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pyactivestorage_amd import storage as pas
    c = 64
    cb = c ** 3 * 4
    path = "/tmp/pyas_prof_dropin.chunks"
    with open(path, "wb") as f:
        for k in range(64):
            f.write((np.arange(c ** 3, dtype=np.float32) + k).tobytes())
    missing = (np.float32(-999.0), None, np.float32(1000.0), np.float32(5e8))
    sel = (slice(0, c, 1),) * 3

    def go(n):
        for k in range(n):
            pas.reduce_chunk(path, (k % 64) * cb, cb, None, None, missing, np.dtype("<f4"), (c, c, c), "C",
                             sel, (0, 1, 2), np.ma.sum)
    go(16)
    pr = cProfile.Profile()
    pr.enable()
    go(200)
    pr.disable()
    os.unlink(path)
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
