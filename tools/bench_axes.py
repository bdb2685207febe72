"""Partial-axis reduction throughput (row f1) on the C3 workload:
1024^3 f32 in 64^3 chunks, _FillValue + valid_min/valid_max, device-resident.
Reports GB/s of pyas_reduce_axes for several axis sets (per chunk, keepdims),
or with --fold of pyas_reduce_axes_grid (the whole-variable box query with
the chunk layers folded in the kernel, what Active runs on resident data).
--shuffle stores the chunks HDF5-byte-shuffled; --only AXES (e.g. "0" or
"0,2") runs one axis set (for per-axis rocprofv3 passes)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("PYAS_TREE"):   # A/B: another build of the package (e.g. the previous round's)
    sys.path.insert(0, os.environ["PYAS_TREE"])


def main():
    import torch
    from pyactivestorage_amd import _lib, engine
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import DeviceBuffer, get_context
    from pyactivestorage_amd.synthetic import chunk_major_device
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    st = torch.cuda.current_stream().cuda_stream
    shape, chunks = (1024, 1024, 1024), (64, 64, 64)
    shuffled = "--shuffle" in sys.argv   # chunks stored HDF5-byte-shuffled
    axis_sets = ((0,), (1,), (2,), (0, 1), (1, 2), (0, 2))
    if "--only" in sys.argv:
        axis_sets = (tuple(int(x) for x in sys.argv[sys.argv.index("--only") + 1].split(",")),)
    for k, arg in enumerate(sys.argv):     # --fold-blocks N: workgroup floor of the in-kernel fold
        if arg == "--fold-blocks":
            ctx.set_fold_min_blocks(int(sys.argv[k + 1]))
    data, offsets, _ = chunk_major_device(torch, shape, chunks, np.float32, dev, fill=-999.0, fill_frac=0.01,
                                          shuffle=shuffled)
    missing = (np.float32(-999.0), None, np.float32(1000.0), np.float32(5e8))
    if "--unmasked" in sys.argv:
        missing = None
    plan = ReductionPlan(ctx, np.float32, chunks, data.data_ptr(), offsets, missing=missing, stream=st,
                         shuffle=4 if shuffled else 0)
    nbytes = data.numel()
    res = {}
    reps = 20

    def timed(fn):
        """Median and min of `reps` launches, each timed with HIP events on
        the launch stream (torch's current stream)."""
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ts)
        return ms[len(ms) // 2] * 1e-3, ms[0] * 1e-3
    if "--fold" in sys.argv:
        grid_n = [s // c for s, c in zip(shape, chunks)]
        for axes in axis_sets:
            g = _lib.Grid()
            g.ndim = 3
            g.axes_mask = sum(1 << a for a in axes)
            for d in range(3):
                g.n_coords[d] = grid_n[d]
                g.out_extent[d] = 1 if d in axes else shape[d]
            n_final = int(np.prod([1 if d in axes else shape[d] for d in range(3)]))
            fin = DeviceBuffer(ctx, n_final * _lib.PARTIAL_NBYTES)
            try:
                engine.reduce_axes_grid(ctx, plan.batch, plan.mask_up.struct, g, fin.ptr, True, st)
            except NotImplementedError as exc:
                res[str(axes)] = {"refused": str(exc)}
                continue
            dt, dmin = timed(lambda: engine.reduce_axes_grid(ctx, plan.batch, plan.mask_up.struct, g, fin.ptr,
                                                            True, st))
            res[str(axes)] = {"ms": round(dt * 1e3, 3), "ms_min": round(dmin * 1e3, 3),
                              "GBps": round(nbytes / dt / 1e9, 1), "outputs": n_final}
            del fin
        print(json.dumps({"workload": "c3 box query, chunk layers folded in-kernel (pyas_reduce_axes_grid)"
                          + (", byte-shuffled chunks" if shuffled else ""), "results": res}))
        return
    # --rec sum|min|max: compact per-output records (pyas_reduce_axes_ex,
    # 8 B per f32 output) instead of the 32-B partials
    rec = 0
    if "--rec" in sys.argv:
        rec = {"sum": _lib.REC_SUM, "min": _lib.REC_MIN, "max": _lib.REC_MAX}[sys.argv[sys.argv.index("--rec") + 1]]
    rb = _lib.rec_nbytes(4, rec)
    for axes in axis_sets:
        n_out = int(np.prod([1 if d in axes else chunks[d] for d in range(3)]))
        out = DeviceBuffer(ctx, len(offsets) * n_out * rb)
        offs = torch.from_numpy(np.arange(len(offsets), dtype=np.int64) * n_out).to(dev)
        mask = 0
        for a in axes:
            mask |= 1 << a
        for _ in range(2):
            engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, mask, offs.data_ptr(), out.ptr, st, rec=rec)
        dt, dmin = timed(lambda: engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, mask,
                                                    offs.data_ptr(), out.ptr, st, rec=rec))
        wbytes = len(offsets) * n_out * rb
        res[str(axes)] = {"ms": round(dt * 1e3, 3), "ms_min": round(dmin * 1e3, 3),
                          "GBps": round(nbytes / dt / 1e9, 1), "frac_read": round(nbytes / dt / 8e12, 4),
                          "GBps_read_write": round((nbytes + wbytes) / dt / 1e9, 1),
                          "outputs_per_chunk": n_out, "write_bytes": wbytes}
        del out
    print(json.dumps({"workload": "c3 partial-axis per-chunk reduce_axes" + (", byte-shuffled chunks" if shuffled else "")
                      + (f", {sys.argv[sys.argv.index('--rec') + 1]} records ({rb} B per output)" if rec else
                         ", 32-B partials"), "results": res}))


if __name__ == "__main__":
    main()
