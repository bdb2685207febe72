"""bench.py's own N-rank launcher, rehearsed on the CPU (gloo, no GPU).

``python bench.py --gpus N`` without WORLD_SIZE must start N rank processes
(before anything touches a GPU) with RANK/LOCAL_RANK/WORLD_SIZE wired, shard
the chunk list into N contiguous ranges, exchange the per-rank partials with
one all-gather and fold them in rank order to the single-rank answer.  It
must never silently run fewer ranks than asked for.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3, 4])
def test_launcher_spawns_n_ranks_and_folds_in_rank_order(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--selftest-launch"],
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    out = lines[0]
    assert out["n_ranks"] == n
    ranks = out["ranks"]
    assert [x["rank"] for x in ranks] == list(range(n))
    assert all(x["env_rank"] == x["rank"] == x["local_rank"] and x["world"] == n for x in ranks)
    # contiguous ranges covering every chunk, in rank order
    assert ranks[0]["range"][0] == 0
    assert all(a["range"][1] == b["range"][0] for a, b in zip(ranks, ranks[1:]))
    assert ranks[-1]["range"][1] == 24
    fin, one = out["final"], out["single"]
    assert fin["count"] == one["count"] and fin["min"] == one["min"] and fin["max"] == one["max"]
    assert fin["sum"] == pytest.approx(one["sum"], rel=1e-12)


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--selftest-launch"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "--gpus 2" in r.stderr


def test_failing_rank_fails_the_launch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--selftest-launch",
                        "--config", "no-such-config"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
