"""Real-size samples of BASELINE.json's C4 and C5 against the oracle
(run by tests/test_gpu_fullsize.py in a fresh process: torch initialises the
GPU first here).

For each sampled chunk the HIP path's per-chunk partial (pyas_reduce_chunks
over bench.py's generator, fill planting and selection table) must equal the
oracle's ``storage.reduce_chunk`` (``storage.py:8-104``: un-shuffle, view,
hyperslab, mask, then ``np.ma.count`` / ``np.ma.sum`` / ``np.ma.min`` /
``np.ma.max``): count, min and max bit for bit, the f32/f64 sum within 1e-6
relative; and the combined total must equal the oracle's
``_from_storage`` combine over the same chunks (``active.py:575-630``):
count, min, max exact, mean within 1e-6.

* C4: 64 chunks of 128^3 f32, byte-shuffled (es 4), _FillValue at 1 %,
  valid_min / valid_max (the chunks at coordinate 0 along dim 2: the
  valid_max of 5e8 masks every chunk beyond).
* C5: 256 chunks of 32^3 f64 with the [16:-16]^3 hyperslab, those with data
  (coordinate 0 along dim 2) in the first four chunk layers: all of them
  half-selected along dim 2, the first layer along dim 0 too, the grid's
  edge chunks along dim 1 as well.

Usage: python -m tests._fullsize_oracle {c4|c5}
"""
import concurrent.futures
import sys

import numpy as np


def main(name):
    import torch  # noqa: F401  (before libpyas_hip: one HIP runtime)

    sys.path.insert(0, ".")
    import bench
    from oracle import storage_ref as ref
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import get_context
    from pyactivestorage_amd.synthetic import chunk_major_device

    # "c4u" / "c5u": the same configs without valid_max, so every chunk
    # holds data and the sums run over full-magnitude values: chunks spread
    # evenly over the whole grid (the masked configs' data sits in the first
    # chunk column along dim 2 only)
    unmasked = name.endswith("u")
    name = name[:-1] if unmasked else name
    cfg = bench.CONFIGS[name]
    dt = np.dtype(cfg["dtype"])
    shape, chunks = cfg["shape"], cfg["chunks"]
    grid = [s // c for s, c in zip(shape, chunks)]
    n_grid = int(np.prod(grid))
    if unmasked:
        ids = sorted({int(x) for x in np.linspace(0, n_grid - 1, 64 if name == "c4" else 256)})
    # valid_max (5e8) masks every chunk beyond the first chunk columns along
    # dim 2 (values i + j*n + k*n^2): sample the chunks that hold data
    elif name == "c4":   # 64 chunks with chunk coordinate 0 along dim 2
        ids = [c for c in range(0, 1024) if c % grid[2] == 0]
    else:              # 256 chunks with coordinate 0 along dim 2, in the first four layers
        ids = [c for c in range(0, 8192) if c % grid[2] == 0]
    ranges = [ids]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    st = torch.cuda.current_stream().cuda_stream
    missing = (dt.type(bench.FILL), None, dt.type(bench.VMIN), None if unmasked else dt.type(bench.VMAX))
    filters = [ref.Shuffle(dt.itemsize)] if cfg["shuffle"] else None
    n_checked = n_partial = 0
    for ids in ranges:
        # each chunk generated on its own: a chunk's bytes (values and fill
        # planting) do not depend on the range it is generated in
        data = torch.cat([chunk_major_device(torch, shape, chunks, dt, dev, chunk_range=(c, c + 1),
                                             fill=bench.FILL, fill_frac=0.01, seed=0,
                                             shuffle=cfg["shuffle"])[0] for c in ids])
        cb = int(np.prod(chunks)) * dt.itemsize
        offsets = np.arange(len(ids), dtype=np.int64) * cb
        rows = [bench.chunk_selections(cfg, shape, c, c + 1) for c in ids]
        table = None if rows[0][0] is None else np.concatenate([r[0] for r in rows])
        counts = np.concatenate([r[1] for r in rows])
        plan = ReductionPlan(ctx, dt, chunks, data.data_ptr(), offsets,
                             shuffle=dt.itemsize if cfg["shuffle"] else 0, sel_table=table,
                             missing=missing, round_to_var=True, stream=st)
        plan.launch(st, chunk_partials=True)
        gpu = plan.read_chunk_partials(st)
        total = plan.read_total(st)[0]
        lo, hi = 0, len(ids)
        host = data.cpu().numpy()

        def sel_of(c):
            if table is None:
                return tuple(slice(0, n) for n in chunks)
            return tuple(slice(int(table[c, d, 0]), int(table[c, d, 0] + table[c, d, 2])) for d in range(3))

        def oracle(c):
            raw = host[c * cb:(c + 1) * cb].tobytes()
            out = {}
            for key, fn in (("sum", np.ma.sum), ("min", np.ma.min), ("max", np.ma.max)):
                tmp, n = ref.reduce_chunk_bytes(raw, None, filters, missing, dt, chunks, "C", sel_of(c),
                                                (0, 1, 2), fn)
                out[key] = tmp
                out["n"] = n
            return out

        with concurrent.futures.ThreadPoolExecutor(max_workers=16) as ex:
            ref_parts = list(ex.map(oracle, range(hi - lo)))
        for c, o in enumerate(ref_parts):
            g = gpu[c]
            n = int(np.asarray(o["n"]).reshape(-1)[0])
            assert int(g["count"]) == n, (name, ids[c], int(g["count"]), n)
            n_partial += int(counts[c]) != int(np.prod(chunks))
            if n == 0:
                continue
            for key in ("min", "max"):
                want = np.asarray(np.ma.getdata(o[key]), dtype=dt).reshape(-1)[0]
                got = np.asarray(g[key], dtype=dt)
                assert got.tobytes() == want.tobytes(), (name, ids[c], key, got, want)
            ws = float(np.asarray(np.ma.getdata(o["sum"])).reshape(-1)[0])
            assert abs(float(g["sum"]) - ws) <= 1e-6 * abs(ws), (name, ids[c], float(g["sum"]), ws)
            n_checked += 1
        # the Active combine over these chunks (active.py:575-630)
        parts = {k: [(o[k], o["n"], (slice(c, c + 1), slice(0, 1), slice(0, 1))) for c, o in enumerate(ref_parts)]
                 for k in ("sum", "min", "max")}
        osum = ref.combine_partials(parts["sum"], (hi - lo, 1, 1), dt, (0, 1, 2), "mean", components=True)
        n = int(np.asarray(osum["n"]).reshape(-1)[0])
        assert int(total["count"]) == n
        omean = float(np.asarray(np.ma.getdata(osum["sum"])).reshape(-1)[0]) / n
        gmean = float(np.asarray(total["sum"], dtype=dt)) / int(total["count"])
        assert abs(gmean - omean) <= 1e-6 * abs(omean), (name, gmean, omean)
        for key in ("min", "max"):
            want = np.asarray(np.ma.getdata(ref.combine_partials(parts[key], (hi - lo, 1, 1), dt, (0, 1, 2),
                                                                 key)), dtype=dt).reshape(-1)[0]
            assert np.asarray(total[key], dtype=dt).tobytes() == want.tobytes(), (name, key)
        del data, plan
        torch.cuda.empty_cache()
    assert n_checked >= (64 if name == "c4" else 256), n_checked
    name += "u" if unmasked else ""
    print(f"fullsize-oracle {name} OK: {n_checked} chunks with data vs storage.reduce_chunk "
          f"({n_partial} partially selected), combine over {sum(len(r) for r in ranges)} chunks")


if __name__ == "__main__":
    main(sys.argv[1])
