"""Run by tests/test_gpu_axes_stream.py::test_auto_choice_at_size in a fresh
process (torch initialises the GPU first).

The configuration pyas_reduce_axes picks by itself at a C3-like size (2048 x
64^3 f32 chunks, 2 GiB, _FillValue + valid range; plain (0,): streamed, 4
items per lane; plain (1,): streamed, 2; shuffled (1,): streamed, 1;
shuffled (0,): dense_col) against PYAS_COL_STREAM=0 (one chunk per
workgroup), byte for byte over all 8 M partials, and three chunks per case
against the oracle's storage.py reduction (activestorage/storage.py:95-104).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from oracle import storage_ref as ref
    from pyactivestorage_amd import _lib, engine
    from pyactivestorage_amd.batch import ReductionPlan
    from pyactivestorage_amd.device import get_context
    from pyactivestorage_amd.synthetic import chunk_major_device
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    ctx = get_context(0)
    shape, chunks = (1024, 1024, 512), (64, 64, 64)
    miss = (np.float32(-999.0), None, np.float32(1000.0), np.float32(5e8))
    pdt = engine.partial_dtype(np.float32)
    sel = tuple(slice(0, n, 1) for n in chunks)
    cb = 64 ** 3 * 4
    n_out = 64 * 64
    for shuffle in (False, True):
        data, offsets, _ = chunk_major_device(torch, shape, chunks, np.float32, dev, fill=-999.0, fill_frac=0.01,
                                              shuffle=shuffle)
        plan = ReductionPlan(ctx, np.float32, chunks, data.data_ptr(), offsets, missing=miss, stream=st,
                             shuffle=4 if shuffle else 0)
        nc = len(offsets)
        offs = torch.from_numpy(np.arange(nc, dtype=np.int64) * n_out).to(dev)
        rf = [ref.Shuffle(4)] if shuffle else None
        for axes in ((0,), (1,)):
            mask = sum(1 << a for a in axes)
            outs = []
            for env in (None, "0"):
                if env is None:
                    os.environ.pop("PYAS_COL_STREAM", None)
                else:
                    os.environ["PYAS_COL_STREAM"] = env
                out = torch.empty(nc * n_out * _lib.PARTIAL_NBYTES, dtype=torch.uint8, device=dev)
                engine.reduce_axes(ctx, plan.batch, plan.mask_up.struct, mask, offs.data_ptr(), out.data_ptr(), st)
                outs.append(out)
            os.environ.pop("PYAS_COL_STREAM", None)
            torch.cuda.synchronize()
            what = f"shuffle={shuffle} axes={axes}"
            assert torch.equal(outs[0], outs[1]), what
            got = outs[0].view(nc, n_out * _lib.PARTIAL_NBYTES)
            for c in (0, 777, nc - 1):
                raw = data[int(offsets[c]):int(offsets[c]) + cb].cpu().numpy().tobytes()
                vals, _ = ref.reduce_chunk_bytes(raw, None, rf, miss, np.dtype("<f4"), chunks, "C", sel, axes, None)
                vm = np.ma.asarray(vals)
                part = np.frombuffer(got[c].cpu().numpy().tobytes(), dtype=pdt)
                cnt = np.ma.count(vm, axis=axes, keepdims=True).reshape(-1)
                np.testing.assert_array_equal(part["count"], cnt, err_msg=what)
                ok = cnt > 0
                for f, fn in (("min", np.ma.min), ("max", np.ma.max)):
                    w = np.ma.getdata(fn(vm, axis=axes, keepdims=True)).reshape(-1)[ok]
                    np.testing.assert_array_equal(part[f][ok].astype(np.float32), w, err_msg=f"{what} chunk {c} {f}")
                wsum = np.ma.filled(vm.astype(np.float64), 0).sum(axis=axes, keepdims=True).reshape(-1)
                np.testing.assert_allclose(part["sum"][ok], wsum[ok], rtol=1e-6, err_msg=what)
            print(f"{what}: {nc} chunks, {nc * n_out} partials identical, 3 chunks match the oracle")
            del outs, got
        del plan, data
    print("axes-stream-auto OK")


if __name__ == "__main__":
    main()
