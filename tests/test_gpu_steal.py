"""HIP WorkStealing parity (needs an MI355X): levels + one balance() per problem.

* every reference-generated fixture (tests/golden/steal_*.npz) is reproduced
  bit-for-bit: levels, the ordered steal requests with their fp64 costs and logged
  occupancies, in-flight accounts, idle / saturated sets after the call;
* larger synthetic C4-shaped problems (distributed_amd/graphs.py:steal_problem) match
  the oracle (oracle/steal.cpp) bit-for-bit, including 4,096 workers;
* edge cases: no stealable task, no thief, every worker a thief.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, STEAL_REFTESTS, steal_files
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
from oracle import oracle
from test_oracle_steal import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = PlacementEngine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", steal_files())
def test_balance_matches_reference_fixture(eng, name):
    p, exp, meta = oracle.load_steal_fixture(os.path.join(GOLDEN, name))
    assert_same(eng.steal_balance(p), exp)


REFPROBLEMS = oracle.load_steal_problems(os.path.join(GOLDEN, STEAL_REFTESTS))


@pytest.mark.parametrize("k", range(len(REFPROBLEMS)), ids=[p[0] for p in REFPROBLEMS])
def test_balance_matches_reference_unit_scenarios(eng, k):
    """test_steal.py:728-777 and :1380-1565 (every permutation, multi-replica who_has)."""
    name, p, exp = REFPROBLEMS[k]
    assert_same(eng.steal_balance(p), exp)


@pytest.mark.parametrize("W,T,hot,seed", [(256, 20000, 0.1, 11), (1024, 60000, 0.05, 12), (4096, 100000, 0.1, 13),
                                          (512, 30000, 0.3, 14)])
def test_balance_matches_oracle_synthetic(eng, W, T, hot, seed):
    p = graphs.steal_problem(W, T, hot_frac=hot, seed=seed)
    out, ref = eng.steal_balance(p), oracle.steal_balance(p)
    assert len(ref["st_task"]) > 0
    assert_same(out, ref)


@pytest.mark.parametrize("W,T,replicas,quantum,seed", [(1024, 40000, 3, 0.0, 21), (1024, 40000, 7, 0.0, 22),
                                                       (2048, 60000, 1, 0.5, 23), (4096, 80000, 4, 0.25, 24)])
def test_balance_thief_runs(eng, W, T, replicas, quantum, seed):
    # the run-ordered thief search: replicated dependencies (<= MAXH distinct holders and
    # beyond) and quantised occupancies (many thieves tied on stack time)
    p = graphs.steal_problem(W, T, seed=seed, replicas=replicas, occ_quantum=quantum)
    out, ref = eng.steal_balance(p), oracle.steal_balance(p)
    assert len(ref["st_task"]) > 0
    assert_same(out, ref)


def test_balance_edge_cases(eng):
    p = graphs.steal_problem(64, 500, seed=3)
    q = dict(p, idle=np.ones(64, np.uint8))  # every worker a thief: nothing to do
    assert_same(eng.steal_balance(q), oracle.steal_balance(q))
    q = dict(p, idle=np.zeros(64, np.uint8))  # no thief
    assert_same(eng.steal_balance(q), oracle.steal_balance(q))
    q = dict(p, fast=np.ones(500, np.uint8))  # nothing stealable
    out = eng.steal_balance(q)
    assert len(out["st_task"]) == 0 and (out["level"] == -1).all()
    assert_same(out, oracle.steal_balance(q))


def test_balance_full_c4(eng):
    """BASELINE.json C4 at full size: WorkStealing.balance over 500k processing tasks on
    4,096 workers x 2 threads (10% hot, zipf 1.5, eight cost-level prefixes), bit-exact
    against the oracle."""
    p = graphs.steal_problem(4096, 500_000, seed=1)
    out, ref = eng.steal_balance(p), oracle.steal_balance(p)
    assert len(ref["st_task"]) > 100_000
    assert_same(out, ref)


@pytest.mark.parametrize("W,T,frac,seed", [(256, 20000, 0.3, 61), (4096, 80000, 0.2, 62), (1024, 40000, 0.8, 63)])
def test_balance_restricted_matches_oracle(eng, W, T, frac, seed):
    """_get_thief with valid_workers / loose restrictions (stealing.py:532-542) at scale;
    the restricted reference fixtures (steal_restricted*.npz) run in the fixture test."""
    p = graphs.steal_problem(W, T, seed=seed, restrict=frac)
    out, ref = eng.steal_balance(p), oracle.steal_balance(p)
    assert len(ref["st_task"]) > 0
    assert_same(out, ref)


@pytest.mark.parametrize("W,T,seed", [(256, 20000, 71), (2048, 60000, 72)])
def test_balance_plugin_state_inputs(eng, W, T, seed):
    """levels_in (the plugin's bins) and in-flight accounts of unconfirmed steals as
    inputs (what GPUWorkStealing passes), plus the visited-victim output."""
    p = graphs.steal_problem(W, T, seed=seed, restrict=0.1)
    rng = np.random.default_rng(seed)
    lv = oracle.steal_balance(p)["level"].copy()
    lv[rng.random(T) < 0.2] = -1  # tasks no longer in a bin
    p["level_in"] = lv
    p["inflight_occ_in"] = np.where(rng.random(W) < 0.3, rng.normal(0, 0.5, W), 0.0)
    p["inflight_tasks_in"] = rng.integers(-2, 3, W).astype(np.int32)
    out, ref = eng.steal_balance(p), oracle.steal_balance(p)
    assert len(ref["st_task"]) > 0
    assert_same(out, ref, keys=tuple(ref))
