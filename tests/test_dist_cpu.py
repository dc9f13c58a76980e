"""CPU, world_size 2 over gloo: bench.py's multi-GPU control plane (clip sharding with no
overlap, barrier, max-over-ranks timing). The data path has no collective to test."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    seeds = bench.clip_seeds(rank, 4)
    allseeds = [None] * world
    dist.all_gather_object(allseeds, seeds)
    dist.barrier()
    dt = bench.max_over_ranks(1.0 + rank, world)
    dist.destroy_process_group()
    q.put((rank, allseeds, dt))
    del torch


@pytest.mark.timeout(120)
def test_two_rank_sharding_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, allseeds, dt in res:
        flat = [s for ss in allseeds for s in ss]
        assert len(flat) == len(set(flat)) == 8  # disjoint shards covering 8 clips
        assert dt == 2.0                          # both ranks see the slowest rank's time
