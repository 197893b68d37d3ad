"""Multi-GPU partitioning of the placement hot path.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on the GPU
box, "gloo" in the CPU tests). What shards and what does not:

* The per-task rows of WorkStealing.balance() — the ``_get_thief`` argmin of
  ``worker_objective`` over the initial thieves, both comm costs and the dependency
  holders of every stealable task (stealing.py:532-542, scheduler.py:3131-3146,
  :3006-3022) — are independent of each other: each rank computes a contiguous slice
  of the stealable positions (``shard_range``) and one all-gather of fixed-size
  records (``gather_rows``) gives every rank all of them.
* The ordered part — the placement replay (one stimulus at a time, every decision
  reading the state the previous one left, scheduler.py:2045-2076) and the walk of
  balance() (:431-503) — does not partition: it runs replicated, every rank on the
  same inputs, and ``replicas_agree`` all-gathers a digest of each rank's output so a
  diverging rank is detected rather than averaged away.
"""
from __future__ import annotations

import hashlib


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Rank ``rank``'s contiguous slice [lo, hi) of ``n`` rows: ceil(n / world) rows per
    rank, the last ranks short (possibly empty)."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError(f"shard_range({n}, {rank}, {world})")
    chunk = -(-n // world)
    lo = min(n, rank * chunk)
    return lo, min(n, lo + chunk)


def chunk_rows(n: int, world: int) -> int:
    return -(-n // world)


def gather_rows(local, n_rows: int, row_bytes: int, group=None):
    """All-gather the ranks' row slices (``local``: a uint8 tensor of chunk_rows(n, world)
    * row_bytes bytes, rank r's rows [shard_range(n, r, world)) first, zero padding after)
    into one tensor whose row i is position i, for i < n_rows."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    chunk = chunk_rows(n_rows, world)
    if local.dtype != torch.uint8 or local.numel() != chunk * row_bytes:
        raise ValueError(f"gather_rows: local slice is {local.numel()} bytes, expected {chunk * row_bytes}")
    if dist.get_backend(group) == "gloo":  # CPU tests; device rows are staged through the host
        host = local.cpu()
        out = torch.empty(world * chunk * row_bytes, dtype=torch.uint8)
        dist.all_gather(list(out.view(world, chunk * row_bytes).unbind(0)), host, group=group)
        return out[: n_rows * row_bytes].to(local.device)
    out = torch.empty(world * chunk * row_bytes, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out[: n_rows * row_bytes]


def output_digest(arrays) -> bytes:
    """sha256 over the raw bytes of a sequence of numpy arrays (one rank's outputs)."""
    h = hashlib.sha256()
    for a in arrays:
        h.update(memoryview(a).cast("B"))
    return h.digest()


def replicas_agree(digest: bytes, device, group=None) -> bool:
    """True iff every rank of ``group`` produced the same 32-byte digest."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    mine = torch.tensor(list(digest), dtype=torch.uint8, device=device)
    allv = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    return all(bool(torch.equal(v, allv[0])) for v in allv)
