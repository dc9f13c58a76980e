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


class _CpuRunner:
    """CPU stand-in for bench.GpuRunner: each step sleeps (rank 1 twice as long) and 'decodes'
    the fixed 220 tokens of every clip of this rank's shard."""

    def setup(self, args, rank, local, barrier):
        import bench

        barrier()
        self.rank, self.B, self.steps = rank, args.batch, 0
        self.seeds = bench.clip_seeds(rank, args.batch)
        self.dt = 0.05 * (1 + rank)

    def sync(self):
        pass

    def step(self):
        import time

        time.sleep(self.dt)
        self.steps += 1

    def events(self, on):
        pass

    def tokens_per_clip(self):
        import bench

        return [bench.MAX_TOKENS + 1] * self.B if self.steps else []

    def profile(self, only=None):
        allc = {"attn_cross": {"ms": 2.0, "launches": 4, "flops": 1e9, "bytes": 8e9},
                "gemm_enc": {"ms": 1.0, "launches": 2, "flops": 2e12, "bytes": 1e8}}
        return {c: v for c, v in allc.items() if not only or c in only}

    def cpu_baseline(self):
        raise AssertionError("world > 1: no cpu baseline")


def _main_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import bench

    run = _CpuRunner()
    out = bench.main(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--batch", "4"], runner=run)
    q.put((rank, out, run.seeds, run.steps))


@pytest.mark.timeout(120)
def test_two_rank_bench_main():
    """bench.main end to end on two gloo ranks: warmup + timed steps + profiled step on every rank,
    the slowest rank's time, the whole-job value over both shards, one JSON line's fields."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_main_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=100) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    seeds = [s for r in res for s in r[2]]
    assert len(seeds) == len(set(seeds)) == 8
    for rank, out, _, steps in res:
        assert steps == 1 + 3  # warmup + timed (the profile pass is the runner's own step)
        assert out["n_gpus"] == 2 and out["steps"] == 3 and out["scaling"] == "weak"
        assert out["config"]["global_batch"] == 8 and out["cpu_baseline"] is None
        # slowest rank: 3 steps x 0.1 s; value = 8 clips x 3 steps x 30 s over that time
        assert 0.3 <= out["ms_per_step"] * 3 / 1e3 < 0.6
        assert abs(out["value"] - 8 * 3 * 30.0 / (out["ms_per_step"] * 3 / 1e3)) < 0.05 * out["value"]
        assert out["roofline"]["kernel_class"] == "attn_cross" and out["roofline"]["bound"] == "hbm"
    assert res[0][1]["ms_per_step"] == res[1][1]["ms_per_step"]  # max over ranks on both
