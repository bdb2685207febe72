"""Where a C3 hyperslab's full reduction spends its time: k_reduce / k_reduce_u
over subsets of the chunks (ReductionPlan + pyas timing events), e.g. the
whole chunks through the selection kernel, only the cut chunks of each kind.

    python tools/probe_reduce_sel.py [--lo 1 --hi 1023] [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lo", type=int, default=1)
    ap.add_argument("--hi", type=int, default=1023)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from pyactivestorage_amd import _lib
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import get_context
    from pyactivestorage_amd.synthetic import chunk_major_device
    cfg = bench.CONFIGS["c3"]
    dt = np.dtype("f4")
    shape, chunks = cfg["shape"], cfg["chunks"]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    data, offsets, _ = chunk_major_device(torch, shape, chunks, dt, dev, fill=bench.FILL, fill_frac=0.01, seed=0)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    missing = (dt.type(bench.FILL), None, dt.type(bench.VMIN), dt.type(bench.VMAX))
    grid = [s // c for s, c in zip(shape, chunks)]
    n = int(np.prod(grid))
    ci = np.stack(np.unravel_index(np.arange(n), grid), axis=1)
    c = np.array(chunks)
    start = np.clip(a.lo - ci * c, 0, c)
    stop = np.clip(a.hi - ci * c, 0, c)
    cnt = np.maximum(stop - start, 0)
    table = np.zeros((n, _lib.MAX_DIMS, 3), dtype=np.int32)
    table[:, :, 1] = 1
    table[:, :, 2] = 1
    table[:, :3, 0] = start
    table[:, :3, 2] = cnt
    whole = (cnt == c).all(axis=1)
    cut = ~whole & (cnt > 0).all(axis=1)
    k2 = cut & (cnt[:, 2] != 64)
    k1 = cut & (cnt[:, 2] == 64) & (cnt[:, 1] != 64)
    k0 = cut & (cnt[:, 2] == 64) & (cnt[:, 1] == 64)
    full_table = np.zeros_like(table)
    full_table[:, :, 1] = 1
    full_table[:, :, 2] = 1
    full_table[:, :3, 2] = c
    cases = {"whole chunks, no table (k_reduce)": (np.arange(n), None),
             "whole chunks, full table (k_reduce_u)": (np.arange(n), full_table),
             f"[{a.lo}:{a.hi}]^3 all": (np.nonzero(cnt.prod(axis=1) > 0)[0], table),
             "its whole chunks": (np.nonzero(whole)[0], table),
             "its cut chunks": (np.nonzero(cut)[0], table),
             "cut in dim 2 (spans)": (np.nonzero(k2)[0], table),
             "cut in dim 1 only (rows)": (np.nonzero(k1)[0], table),
             "cut in dim 0 only (contiguous)": (np.nonzero(k0)[0], table)}
    res = {}
    for name, (idx, tab) in cases.items():
        if not len(idx):
            continue
        plan = ReductionPlan(ctx, dt, chunks, data.data_ptr(), offsets[idx],
                             sel_table=None if tab is None else tab[idx], index_pool=np.zeros(1, np.int32),
                             missing=missing, round_to_var=True, stream=st)
        for _ in range(3):
            plan.launch(st, chunk_partials=False)
        torch.cuda.synchronize()
        _lib.check(ctx.lib.pyas_timing_enable(ctx.handle, a.reps), "timing_enable")
        for _ in range(a.reps):
            plan.launch(st, chunk_partials=False)
        torch.cuda.synchronize()
        ms = (ctypes.c_float * a.reps)()
        nrec = ctypes.c_int32(0)
        _lib.check(ctx.lib.pyas_timing_read(ctx.handle, ms, a.reps, ctypes.byref(nrec)), "timing_read")
        _lib.check(ctx.lib.pyas_timing_enable(ctx.handle, 0), "timing_disable")
        kms = float(np.median(np.array(ms[: nrec.value])))
        sel = int((cnt[idx].prod(axis=1) if tab is not None else np.full(len(idx), 64 ** 3)).sum()) * 4
        res[name] = {"chunks": int(len(idx)), "bytes": sel, "kernel_ms": round(kms, 4),
                     "TBps": round(sel / kms / 1e9, 3), "frac": round(sel / kms / 1e9 / 8.0, 4)}
        print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps({"probe": "reduce_sel", "lo": a.lo, "hi": a.hi, "spans": os.environ.get("PYAS_SPANS", "1"),
                      "results": res}))


if __name__ == "__main__":
    main()
