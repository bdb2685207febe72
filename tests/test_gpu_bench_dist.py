"""bench.py's N-rank body on the GPU box before an 8-GPU node runs it
(row e): ``--gpus 2 --dist-backend gloo`` starts two ranks that share the
box's GPU, each reducing its own shard (weak C3-shaped headline, strong
C4/C5-shaped extras at small sizes), exchanges the 32-byte rank partials
(staged through host memory for gloo) and the per-chunk partials as
tensors, and self-checks the sharded result against a single-rank combine
of every chunk partial (active.py:557-598 has no multi-process mode; its
thread pool's combine is the reference)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_bench_ranks_gloo_share_one_gpu(gpu, world):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
           "--config", "t3", "--extra", "t4,t5", "--steps", "3", "--warmup", "1", "--extra-steps", "3",
           "--cpu-chunks", "0", "--host-inclusive", "0", "--file-inclusive", "0"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == world and line["config"]["exchange"] == "gloo"
    assert len(line["per_rank"]["kernel_ms"]) == world and all(k > 0 for k in line["per_rank"]["kernel_ms"])
    assert len(line["per_rank"]["exchange_combine_ms"]) == world
    assert line["selfcheck"]["ok"], line["selfcheck"]
    assert sum(line["per_rank"]["chunks"]) == line["config"]["chunks_total"]
    for k in ("t4_strong", "t5_strong"):
        ex = line["extra"][k]
        assert len(ex["per_rank"]["kernel_ms"]) == world and ex["selfcheck"]["ok"], (k, ex["selfcheck"])


def test_bench_refuses_more_ranks_than_gpus(gpu):
    """nccl (one GPU per rank): the launcher counts GPUs from sysfs without
    touching them and refuses --gpus beyond what the box has."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "1", "--warmup", "0"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr
