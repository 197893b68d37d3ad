"""The sharded WorkStealing.balance() on the device (needs an MI355X), DESIGN.md §8.

* Two engines, one slice of the thief rows each (dgp_steal_thief_rows), exchange the
  packed 128-byte records through device buffers and both finish the walk
  (dgp_steal_run): each result equals the one-shot dgp_steal_balance and the oracle.
* Two processes on the one GPU, a gloo group between them (RCCL needs one GPU per
  rank; the box has one): ``PlacementEngine.steal_balance(p, group)`` end to end, both
  ranks bit-exact against the oracle.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from distributed_amd import graphs, shard
from distributed_amd.engine import PlacementEngine
from oracle import oracle
from test_oracle_steal import assert_same

pytestmark = pytest.mark.gpu


def _sliced(engines, p):
    import torch

    args = [e._steal_args(p) for e in engines]
    ns = []
    for e, (inputs, *_rest) in zip(engines, args):
        n = C.c_int64(0)
        e._check(e.lib.dgp_steal_load(e.h, *inputs, C.byref(n)), "dgp_steal_load")
        ns.append(int(n.value))
    assert len(set(ns)) == 1
    n, world = ns[0], len(engines)
    rb = int(engines[0].lib.dgp_steal_row_bytes())
    assert rb == 128
    full = torch.zeros(shard.chunk_rows(n, world) * world * rb, dtype=torch.uint8, device="cuda")
    for r, e in enumerate(engines):
        lo, hi = shard.shard_range(n, r, world)
        e._check(e.lib.dgp_steal_thief_rows(e.h, lo, hi), "rows")
        if hi > lo:
            e._check(e.lib.dgp_steal_pack_rows(e.h, lo, hi, C.c_void_p(full.data_ptr() + lo * rb)), "pack")
    torch.cuda.synchronize()
    outs = []
    for e, (inputs, outputs, out, cnt, keep) in zip(engines, args):
        if n:
            e._check(e.lib.dgp_steal_unpack_rows(e.h, 0, n, C.c_void_p(full.data_ptr())), "unpack")
        e._check(e.lib.dgp_steal_run(e.h, *outputs), "run")
        outs.append(e._steal_result(out, cnt))
    return outs


@pytest.mark.parametrize("W,T,seed", [(256, 20000, 31), (4096, 60000, 32), (64, 3, 33)])
def test_two_engines_exchange_rows(W, T, seed):
    p = graphs.steal_problem(W, T, seed=seed)
    ref = oracle.steal_balance(p)
    with PlacementEngine(0) as a, PlacementEngine(0) as b, PlacementEngine(0) as one:
        assert_same(one.steal_balance(p), ref)
        for out in _sliced([a, b], p):
            assert_same(out, ref)
        for out in _sliced([a, b, one], p):  # three slices, one engine reused
            assert_same(out, ref)


def test_row_calls_check_state_and_ranges():
    with PlacementEngine(0) as e:
        assert e.lib.dgp_steal_thief_rows(e.h, 0, 1) != 0  # no dgp_steal_load yet
        p = graphs.steal_problem(64, 500, seed=5)
        inputs, outputs, out, cnt, keep = e._steal_args(p)
        n = C.c_int64(0)
        e._check(e.lib.dgp_steal_load(e.h, *inputs, C.byref(n)), "load")
        assert e.lib.dgp_steal_thief_rows(e.h, 0, int(n.value) + 1) != 0
        assert e.lib.dgp_steal_thief_rows(e.h, 2, 1) != 0
        assert e.lib.dgp_steal_pack_rows(e.h, 0, 1, None) != 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        torch.cuda.set_device(0)
        p = graphs.steal_problem(1024, 40000, seed=41)
        with PlacementEngine(0) as e:
            out = e.steal_balance(p, group=dist.group.WORLD)
        ref = oracle.steal_balance(p)
        ok = all(np.array_equal(np.asarray(out[k]), np.asarray(ref[k])) for k in ref)
        q.put((rank, ok, len(ref["st_task"])))
    finally:
        dist.destroy_process_group()


def test_two_processes_sharded_balance():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert all(n > 0 for _, _, n in res)
