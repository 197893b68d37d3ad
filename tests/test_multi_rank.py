"""The N>1 path of bench.py on the CPU: world_size 2 over gloo (127.0.0.1).

The placement path does not shard ("replicas only"): every rank replays
its own copy of the workload, and the job's time is the slowest rank's. This test runs
that protocol with two gloo ranks, using the oracle as each rank's CPU stand-in for the
device replay: both replicas must produce identical placements, and ``reduce_max`` must
return the maximum over ranks on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from distributed_amd import graphs
from oracle import oracle


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = graphs.random_dag(2000, 32, seed=3)  # every rank: the same replica
        out = oracle.replay(g, bench.CONFIG, snapshots=False)
        digest = int(np.bitwise_xor.reduce(out["pl_task"].astype(np.int64) * 1315423911 + out["pl_worker"]))
        fake_elapsed = 1.0 + rank  # rank 1 is the slow one
        slowest = bench.reduce_max(fake_elapsed, dist, device="cpu")
        dist.barrier()
        q.put((rank, digest, len(out["pl_task"]), slowest))
    finally:
        dist.destroy_process_group()


def test_two_rank_replicas_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    digests = {r[1] for r in res}
    assert len(digests) == 1, "replicas disagree"
    assert all(r[2] == 2000 for r in res)
    assert all(r[3] == pytest.approx(2.0) for r in res), res


def test_reduce_max_single_process():
    assert bench.reduce_max(3.5, None) == 3.5
