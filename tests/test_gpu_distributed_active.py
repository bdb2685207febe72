"""Row (e) at the API level: ``Active(..., group=...)`` under torch.distributed.

Each rank reads and reduces a contiguous range of the query's chunks on the
GPU; the per-rank partial grids are all-gathered and folded in rank order on
the device.  The reference has no multi-process mode (its parallelism is the
thread pool of active.py:557-598), so the expectation is the single-process
result of the same queries: counts, masks, min and max exact, sums and means
within 1e-6 relative (the chunk partials are associated differently).  The
ranks here share the box's one GPU and exchange over gloo; the RCCL path is
exercised by bench.py --force-dist.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests import _dist_active as D

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_active_matches_local(gpu, tmp_path, world):
    want = D.run_queries()
    out = tmp_path / "dist.npz"
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(D.ROOT, "tests", "_dist_active.py"),
                                       str(out)], env=env, cwd=D.ROOT))
    for p in procs:
        assert p.wait(timeout=100) == 0
    got = np.load(out)
    for k in range(len(D.QUERIES)):
        wd, wm = want[f"q{k}_data"], want[f"q{k}_mask"]
        gd, gm = got[f"q{k}_data"], got[f"q{k}_mask"]
        assert gd.shape == wd.shape and gd.dtype == wd.dtype, k
        np.testing.assert_array_equal(gm, wm, err_msg=f"query {k} mask")
        method = D.QUERIES[k][0]
        if method in ("min", "max"):
            np.testing.assert_array_equal(gd[~wm], wd[~wm], err_msg=f"query {k}")
        else:
            np.testing.assert_allclose(gd[~wm], wd[~wm], rtol=1e-6, err_msg=f"query {k}")
    for k in range(len(D.ZQUERIES)):
        wd, wm = want[f"z{k}_data"], want[f"z{k}_mask"]
        gd, gm = got[f"z{k}_data"], got[f"z{k}_mask"]
        np.testing.assert_array_equal(gm, wm, err_msg=f"zero query {k} mask")
        assert (wd[~wm] == 0).sum() > 0, k
        assert gd[~wm].tobytes() == wd[~wm].tobytes(), f"zero query {k}: bytes (zero signs) differ"
