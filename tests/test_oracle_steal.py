"""The stealing oracle (oracle/steal.cpp) against the reference's own outputs.

The fixtures were produced by the reference ``WorkStealing`` plugin over a reference
``SchedulerState`` (tests/golden/gen_steal.py). Every task's cost level
(``steal_time_ratio``, distributed/stealing.py:241-277) and the complete result of one
``balance()`` (stealing.py:401-503) must match bit-for-bit: the ordered steal requests
(task, victim, thief, level, fp64 cost, fp64 victim / thief occupancies as logged), the
per-worker in-flight occupancy (fp64) and task deltas, and the idle / saturated sets
after the call. The five cases cover the three victim-selection paths: fewer than 20
saturated workers (sorted list), 20 or more (the live saturated set, re-read per
level), and none saturated (``topk`` of combined occupancy).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, STEAL_REFTESTS, steal_files
from oracle import oracle

STEAL_KEYS = ("level", "st_task", "st_victim", "st_thief", "st_level", "st_cost", "st_occ_victim", "st_occ_thief",
              "inflight_occ", "inflight_tasks", "idle_after", "sat_after")


def assert_same(out, exp, keys=STEAL_KEYS):
    for k in keys:
        a, b = np.asarray(out[k]), np.asarray(exp[k])
        assert a.shape == b.shape, (k, a.shape, b.shape)
        if a.dtype.kind == "f":  # bit-exact, not just ==
            a, b = a.view(np.int64), b.view(np.int64)
        bad = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
        assert len(bad) == 0, f"{k}: {len(bad)} mismatches, first at {bad[0]}"


def test_steal_fixtures_present():
    assert len(steal_files()) >= 5


@pytest.mark.parametrize("name", steal_files())
def test_oracle_matches_reference_balance(name):
    p, exp, meta = oracle.load_steal_fixture(os.path.join(GOLDEN, name))
    assert_same(oracle.steal_balance(p), exp)


def test_fixtures_cover_victim_paths():
    n_sat = {}
    for name in steal_files():
        p, exp, meta = oracle.load_steal_fixture(os.path.join(GOLDEN, name))
        n_sat[name] = int(p["sat"].sum())
    assert any(v == 0 for v in n_sat.values()), n_sat          # topk path
    assert any(0 < v < 20 for v in n_sat.values()), n_sat      # sorted list
    assert any(v >= 20 for v in n_sat.values()), n_sat         # live saturated set


def test_levels_cover_range():
    seen = set()
    for name in steal_files():
        p, exp, meta = oracle.load_steal_fixture(os.path.join(GOLDEN, name))
        seen |= set(int(x) for x in exp["level"])
    assert 0 in seen and len(seen - {-1}) >= 10, sorted(seen)


REFPROBLEMS = oracle.load_steal_problems(os.path.join(GOLDEN, STEAL_REFTESTS))


@pytest.mark.parametrize("k", range(len(REFPROBLEMS)), ids=[p[0] for p in REFPROBLEMS])
def test_oracle_matches_reference_unit_scenarios(k):
    """The reference's own balance scenarios (test_steal.py:728-777 test_balance and the
    dependency-balance family :1380-1565 over every worker permutation, with replicas on
    several workers): the first balance() of each, bit-exact."""
    name, p, exp = REFPROBLEMS[k]
    assert_same(oracle.steal_balance(p), exp)
