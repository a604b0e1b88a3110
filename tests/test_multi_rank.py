"""CPU, world size 2 on gloo: the bench's multi-rank path.

Each rank times its own steps between barriers; the reported time is the
MAX over ranks (all_reduce MAX), and the whole-job value counts every
rank's frames over that time.  Ranks own different frames (weak scaling,
no data-path collective)."""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = {"timed": 0, "untimed": 0}

        def step(record=False):
            calls["timed" if record else "untimed"] += 1
            time.sleep(0.02 * (rank + 1))  # rank 1 is the slow one

        elapsed = bench.timed_region(step, 5, 2, world, lambda: None, torch.device("cpu"))
        rgba, mb, co, _ = bench.make_inputs(2, rank, torch.device("cpu"))
        out[rank] = (elapsed, calls["timed"], calls["untimed"], int(rgba.to(torch.int64).sum()), int(mb.to(torch.int64).sum()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_gloo():
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    (e0, t0, u0, px0, mb0), (e1, t1, u1, px1, mb1) = res[0], res[1]
    assert (t0, u0) == (5, 2) and (t1, u1) == (5, 2)  # exactly K timed, W untimed
    assert e0 == e1  # both ranks report the MAX
    assert e0 >= 5 * 0.04  # ... which is the slow rank's time
    assert px0 != px1 and mb0 != mb1  # each rank owns different frames
    v = bench.aggregate_mpix_s(world, 64, 5, e0)
    assert v == pytest.approx(2 * 64 * 1920 * 1080 * 5 / e0 / 1e6)
