"""HIP engine parity (needs an MI355X).

* every golden fixture (produced by the reference SchedulerState itself) must be
  reproduced bit-for-bit: the placement log (task, worker, comm bytes, fp64
  objective, ws.nbytes, route) and every per-round worker snapshot;
* larger synthetic graphs must match the oracle (oracle/replay.cpp) bit-for-bit.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from oracle import oracle

pytestmark = pytest.mark.gpu

PL_KEYS = ("pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")
ROUND_KEYS = ("round_nplaced", "round_occ", "round_wnbytes", "round_nproc", "round_idle", "round_sat",
              "round_itc", "round_nqueued")


def assert_same(out, exp, keys):
    for k in keys:
        a, b = np.asarray(out[k]), np.asarray(exp[k])
        assert a.shape == b.shape, (k, a.shape, b.shape)
        bad = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
        assert len(bad) == 0, (f"{k}: {len(bad)} mismatches, first at flat index {bad[0]}: "
                               f"{a.reshape(-1)[bad[0]]!r} vs {b.reshape(-1)[bad[0]]!r}")


@pytest.fixture(scope="module")
def engine_cls():
    from distributed_amd.engine import PlacementEngine

    return PlacementEngine


@pytest.mark.parametrize("name", golden_files())
def test_engine_matches_reference_fixture(engine_cls, name):
    g, cfg, exp, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    R = len(exp["round_nplaced"]) + 2
    with engine_cls(0) as eng:
        eng.load(g, cfg, snapshots=R)
        eng.replay()
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("sat", [1.1, "inf"])
@pytest.mark.parametrize("n,w", [(100_000, 1024), (30_000, 4096)])
def test_engine_matches_oracle_random_dag(engine_cls, n, w, sat):
    from distributed_amd import graphs

    g = graphs.random_dag(n, w, seed=42)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": sat}
    ref = oracle.replay(g, cfg, snapshots=False)
    with engine_cls(0) as eng:
        eng.load(g, cfg)
        eng.replay()
        out = eng.placements()
    assert_same(out, ref, PL_KEYS)


def test_engine_matches_oracle_tree_reduce(engine_cls):
    from distributed_amd import graphs

    g = graphs.map_tree_reduce(200_000, 2048, seed=3)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    ref = oracle.replay(g, cfg, snapshots=False)
    with engine_cls(0) as eng:
        eng.load(g, cfg)
        eng.replay()
        out = eng.placements()
    assert_same(out, ref, PL_KEYS)


def test_engine_full_c5_digest(engine_cls):
    """BASELINE.json C5 at full size (10M tasks x 16,384 workers): the device's placement
    log equals the oracle's, pinned by digest (tests/golden/c5_full_digest.json,
    tools/c5_digest.py); every task is placed exactly once."""
    import json

    from distributed_amd import graphs

    pin = json.load(open(os.path.join(GOLDEN, "c5_full_digest.json")))
    g = graphs.map_tree_reduce(pin["n_map"], pin["n_workers"])
    with engine_cls(0) as eng:
        eng.load(g, pin["config"])
        eng.replay()
        out = eng.placements()
    assert len(out["pl_task"]) == pin["n_placements"] == g["n_tasks"]
    assert np.array_equal(np.sort(out["pl_task"]), np.arange(g["n_tasks"]))
    assert graphs.placement_digest(out) == pin["digest"]


@pytest.mark.parametrize("sat,restricted", [(1.1, False), ("inf", False), (1.1, True)],
                         ids=["sat1.1", "satinf", "restricted"])
def test_engine_full_c3_shuffle(engine_cls, sat, restricted):
    """BASELINE.json C3 at full size: P = 66,666 partitions (3P + 1 = 200k tasks: inputs,
    shuffle-transfer, one barrier of fan-in P, unpack tasks with _rootish False) on 512
    workers, bit-exact against the oracle; also with the unpacks restricted to their
    range-sharded worker (restrict_task, shuffle/_scheduler_plugin.py:101-115)."""
    from distributed_amd import graphs

    g = graphs.shuffle_graph(66_666, 512, restricted=restricted)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": sat}
    ref = oracle.replay(g, cfg, snapshots=False)
    with engine_cls(0) as eng:
        eng.load(g, cfg)
        eng.replay()
        out = eng.placements()
    assert len(out["pl_task"]) == g["n_tasks"]
    assert_same(out, ref, PL_KEYS)


def test_engine_full_c2(engine_cls):
    """BASELINE.json C2 at full size (1M tasks x 1,024 workers, saturation 1.1): the whole
    placement log bit-exact against the oracle."""
    from distributed_amd import graphs

    g = graphs.random_dag(1_000_000, 1024, seed=0)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    ref = oracle.replay(g, cfg, snapshots=False)
    with engine_cls(0) as eng:
        eng.load(g, cfg)
        eng.replay()
        out = eng.placements()
    assert len(out["pl_task"]) == g["n_tasks"]
    assert_same(out, ref, PL_KEYS)


@pytest.mark.parametrize("window", [32, 64])
@pytest.mark.parametrize("name", ["c2mini_sat1.1.npz", "c2var_sat1.1.npz", "restr_sat1.1.npz", "c3mini_sat1.1.npz"])
def test_both_window_builds_match_fixture(engine_cls, name, window):
    """Each fixture on BOTH stream-kernel builds, forced (dgp_set_window: 32-slot window with
    wait-in-place claims; 64 slots, no wait-in-place): the auto choice runs restricted graphs
    only on the 64-slot build and C2-shaped ones only on the 32-slot one, so each build also
    runs the other's shapes here."""
    g, cfg, exp, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    R = len(exp["round_nplaced"]) + 2
    with engine_cls(0, window=window) as eng:
        eng.load(g, cfg, snapshots=R)
        eng.replay()
        out = eng.placements()
        out.update(eng.snapshots(R))
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)


@pytest.mark.parametrize("window", [32, 64])
def test_both_window_builds_match_oracle_c3_restricted(engine_cls, window):
    from distributed_amd import graphs

    g = graphs.shuffle_graph(6_000, 128, restricted=True)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    ref = oracle.replay(g, cfg, snapshots=False)
    with engine_cls(0, window=window) as eng:
        eng.load(g, cfg)
        eng.replay()
        out = eng.placements()
    assert_same(out, ref, PL_KEYS)
