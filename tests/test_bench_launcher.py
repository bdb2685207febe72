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


def test_hung_rank_ends_the_launch_within_the_wall_limit():
    """one rank that never joins the exchange (it sleeps
    an hour) must not hang the run.  The launcher's wall limit stops every
    rank, names the ones still running and exits 124 well inside the bound."""
    import time
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--selftest-launch", "--selftest-hang-rank", "1",
                        "--launch-timeout", "25", "--dist-timeout", "600"],
                       env=_env(), capture_output=True, text=True, timeout=200)
    took = time.monotonic() - t0
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert "wall limit" in r.stderr and "1" in r.stderr.split("ranks", 1)[1].split("still", 1)[0]
    assert took < 25 + 60, took


def test_failing_rank_is_named():
    """A rank that exits non-zero fails the launch with its status, is named,
    and the ranks left waiting in the exchange are stopped."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--selftest-launch", "--selftest-fail-rank", "2",
                        "--launch-timeout", "100"], env=_env(), capture_output=True, text=True, timeout=200)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "bench.py: rank 2 exited with status 3" in r.stderr
