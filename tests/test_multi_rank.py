"""The N>1 protocol on the CPU: world_size 2 over gloo (127.0.0.1), DESIGN.md §8.

* The sharded part — the per-task thief rows of balance() — is split by
  ``shard.shard_range`` and merged by ``shard.gather_rows`` (one all-gather of 128-byte
  records). Here each rank builds its slice with a numpy stand-in of the row producer
  (the device kernel needs a GPU; tests/test_gpu_shard.py runs the real one) and the
  merged buffer must equal the one a single process builds, byte for byte, for row
  counts that divide evenly, do not, and leave a rank empty.
* The replicated part — the ordered replay / walk — is checked by ``replicas_agree``
  (all-gathered output digests) and timed by ``bench.reduce_max``.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from distributed_amd import shard

ROW = 128


def stand_in_rows(lo, hi):
    """Deterministic per-position records (what k_best_thief + k_pack_rows produce per
    stealable position): a row depends only on its position."""
    pos = np.arange(lo, hi, dtype=np.int64)
    rec = np.zeros((hi - lo, ROW // 8), np.int64)
    rec[:, 0] = pos * 2654435761 % 4096  # "thief"
    rec[:, 1] = pos ** 2 % 1000003
    rec[:, 2:] = (pos[:, None] * np.arange(1, ROW // 8 - 1)) % 251
    return rec.view(np.uint8).reshape(-1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for n in (0, 1, 7, 1000, 1001):
            lo, hi = shard.shard_range(n, rank, world)
            local = np.zeros(shard.chunk_rows(n, world) * ROW, np.uint8)
            local[: (hi - lo) * ROW] = stand_in_rows(lo, hi)
            full = shard.gather_rows(torch.from_numpy(local), n, ROW)
            res[n] = bool(np.array_equal(full.numpy(), stand_in_rows(0, n)))
        same = shard.replicas_agree(shard.output_digest([np.arange(10)]), "cpu")
        differ = shard.replicas_agree(shard.output_digest([np.arange(10) + rank]), "cpu")
        slowest = bench.reduce_max(1.0 + rank, dist, device="cpu")
        total = bench.reduce_sum(10.0 + rank, dist, device="cpu")  # distinct per-rank work adds up
        dist.barrier()
        q.put((rank, res, same, differ, (slowest, total)))
    finally:
        dist.destroy_process_group()


def test_two_rank_row_exchange_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, merged, same, differ, slowest in res:
        assert all(merged.values()), (rank, merged)
        assert same and not differ
        assert slowest == (pytest.approx(2.0), pytest.approx(21.0))


@pytest.mark.parametrize("n", [0, 1, 5, 8, 9, 1000, 1001])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(n, world):
    spans = [shard.shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and a <= b
    assert all(b - a <= shard.chunk_rows(n, world) for a, b in spans)


def test_shard_range_rejects_bad_args():
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)
    with pytest.raises(ValueError):
        shard.shard_range(-1, 0, 1)


def test_reduce_max_single_process():
    assert bench.reduce_max(3.5, None) == 3.5
    assert bench.reduce_sum(3.5, None) == 3.5
