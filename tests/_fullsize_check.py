"""Child-process body of tests/test_gpu_fullsize.py (torch must initialise
the GPU before libpyas_hip in a process, so each config runs in a fresh
interpreter).  Usage: python -m tests._fullsize_check c3"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SUM_RTOL = 1e-6   # BASELINE.json north star: <= 1e-6 relative for f32/f64 sum/mean


def _torch_reference(torch, buf, cfg, sels, missing, n_chunks):
    """count, f64 sum, min, max of the selected unmasked elements, on the
    device with plain torch ops (buf holds unshuffled chunk-major bytes)."""
    tdt = torch.float32 if cfg["dtype"] == "f4" else torch.float64
    chunks = cfg["chunks"]
    celems = int(np.prod(chunks))
    vals = buf.view(tdt)[: n_chunks * celems].view(n_chunks, *chunks)
    dev = buf.device
    batch = max(1, (256 << 20) // (celems * np.dtype(cfg["dtype"]).itemsize))
    idx = [torch.arange(c, device=dev).view([1] + [-1 if d == k else 1 for d in range(3)])
           for k, c in enumerate(chunks)]
    count, total = 0, 0.0
    mn, mx = float("inf"), float("-inf")
    for b0 in range(0, n_chunks, batch):
        b1 = min(n_chunks, b0 + batch)
        v = vals[b0:b1]
        ok = torch.ones_like(v, dtype=torch.bool)
        if missing[0] is not None:
            ok &= v != float(missing[0])
            ok &= v >= float(missing[2])
            ok &= v <= float(missing[3])
        if sels is not None:
            start = torch.from_numpy(sels[b0:b1, :3, 0].astype(np.int64)).to(dev)
            cnt = torch.from_numpy(sels[b0:b1, :3, 2].astype(np.int64)).to(dev)
            for k in range(3):
                s = start[:, k].view(-1, 1, 1, 1)
                e = s + cnt[:, k].view(-1, 1, 1, 1)
                ok &= (idx[k] >= s) & (idx[k] < e)
        count += int(ok.sum().item())
        total += float(torch.where(ok, v.double(), 0.0).sum().item())
        mn = min(mn, float(torch.where(ok, v, float("inf")).min().item()))
        mx = max(mx, float(torch.where(ok, v, float("-inf")).max().item()))
    return count, total, mn, mx


def _reduce(ctx, dt, cfg, buf, offsets, sels, missing, shuffled, stream):
    from pyactivestorage_amd.batch import ReductionPlan
    plan = ReductionPlan(ctx, dt, cfg["chunks"], buf.data_ptr(), offsets,
                         shuffle=dt.itemsize if shuffled else 0, sel_table=sels,
                         missing=missing, round_to_var=True, stream=stream)
    plan.launch(stream, chunk_partials=False)
    return plan.read_total(stream)[0]


def check(name):
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")   # torch's HIP runtime first
    import bench
    from pyactivestorage_amd.device import get_context
    gpu = get_context(0)
    from pyactivestorage_amd.synthetic import chunk_major_device
    cfg = bench.CONFIGS[name]
    dt = np.dtype(cfg["dtype"])
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    shape = tuple(cfg["shape"])
    n_all = int(np.prod([s // c for s, c in zip(shape, cfg["chunks"])]))
    sels, counts = bench.chunk_selections(cfg, shape, 0, n_all)
    missing = ((dt.type(bench.FILL), None, dt.type(bench.VMIN), dt.type(bench.VMAX))
               if cfg["masked"] else (None, None, None, None))
    fill = bench.FILL if cfg["masked"] else None
    frac = 0.01 if cfg["masked"] else 0.0
    plain, offsets, _ = chunk_major_device(torch, shape, cfg["chunks"], dt, dev, fill=fill,
                                           fill_frac=frac, seed=0, shuffle=False)
    torch.cuda.synchronize()
    got = _reduce(gpu, dt, cfg, plain, offsets, sels, missing, False, stream)
    want_n, want_sum, want_min, want_max = _torch_reference(torch, plain, cfg, sels, missing, n_all)
    assert int(got["count"]) == want_n
    assert want_n > 0
    assert float(got["min"]) == want_min and float(got["max"]) == want_max
    assert abs(float(got["sum"]) - want_sum) <= SUM_RTOL * abs(want_sum)

    # additivity over a split of the chunk list (two independent launches)
    h = n_all // 3
    parts = [_reduce(gpu, dt, cfg, plain, offsets[a:b], None if sels is None else sels[a:b], missing,
                     False, stream) for a, b in ((0, h), (h, n_all))]
    assert sum(int(p["count"]) for p in parts) == int(got["count"])
    assert min(float(p["min"]) for p in parts) == float(got["min"])
    assert max(float(p["max"]) for p in parts) == float(got["max"])
    psum = sum(float(p["sum"]) for p in parts)
    assert abs(psum - float(got["sum"])) <= SUM_RTOL * abs(float(got["sum"]))

    if cfg["shuffle"]:
        del plain
        torch.cuda.empty_cache()
        shuf, offsets_s, _ = chunk_major_device(torch, shape, cfg["chunks"], dt, dev, fill=fill,
                                                fill_frac=frac, seed=0, shuffle=True)
        torch.cuda.synchronize()
        got_s = _reduce(gpu, dt, cfg, shuf, offsets_s, sels, missing, True, stream)
        # the un-shuffle changes which lane adds which element (sum order), not the set
        assert int(got_s["count"]) == int(got["count"])
        assert float(got_s["min"]) == float(got["min"]) and float(got_s["max"]) == float(got["max"])
        assert abs(float(got_s["sum"]) - float(got["sum"])) <= SUM_RTOL * abs(float(got["sum"]))
        del shuf
    torch.cuda.empty_cache()
    print(f"fullsize {name} OK: count={int(got['count'])} sum={float(got['sum']):.9e} "
          f"min={float(got['min'])} max={float(got['max'])}", flush=True)


if __name__ == "__main__":
    check(sys.argv[1])
