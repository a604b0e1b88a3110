"""CPU: `python bench.py --gpus N` starts N ranks itself,
and its N > 1 gather to rank 0 delivers every rank's outputs.

The launcher path is bench.py's own: with --gpus 2 and no WORLD_SIZE in the
environment, bench.py runs torch.distributed.run in a child process (the
parent never opens a device), each rank joins the process group and rank 0
reports how many joined.  --launcher-check swaps the GPU pipeline for an empty
step on gloo, so this runs without a GPU; the timing / MAX-over-ranks logic it
exercises is tests/test_multi_rank.py's."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [1, 2])
def test_gpus_flag_launches_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launcher-check",
                        "--steps", "3", "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["ranks_joined"] == n
    assert rec["steps"] == 3 and rec["warmup"] == 1 and rec["value"] is None
    if n > 1:  # main()'s N > 1 gather (shard.timed_gather_to_root): every rank's outputs reach rank 0 intact
        g = rec["gather"]
        assert g["ok"] and g["bytes_to_root"] == g["bytes_per_rank"] * (n - 1) and g["bytes_per_rank"] > 0
    else:
        assert rec["gather"] is None


@pytest.mark.timeout(120)
def test_world_size_must_match_gpus():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launcher-check"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 2 and "--gpus is 2" in r.stderr
