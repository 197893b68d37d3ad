"""bench.py's C4 balance() leg runs GPUWorkStealing's product path (``balance_plan``: the
plugin's StealRows -> problem -> device) on a scheduler-free stand-in of the plugin state
(tools/steal_standin.py). On CPU: the stand-in's problem, put in the device's walk
order (dgp_steal_order's sort), is the C4 problem itself, and the oracle gives the same
requests on both (the task index of each request mapped through the row slots)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from distributed_amd import graphs  # noqa: E402
from steal_standin import plugin_from_problem  # noqa: E402
from distributed_amd.stealing import ordered_problem
from oracle import oracle


def _same_problem(p, q, T):
    for k in ("nthreads", "occ", "nproc", "wnbytes", "idle", "sat", "victim", "duration", "fast", "level_in"):
        assert np.array_equal(np.asarray(p[k]), np.asarray(q[k])), k
    for k in ("total_occ", "total_nthreads", "bandwidth"):
        assert p[k] == q[k], k
    hp, hi = (p["holder_ptr"], p["holder_idx"]) if "holder_ptr" in p else oracle.holder_csr(p["data_holder"])

    def rows(x, ptr, idx, nb, gnb):
        out = []
        for t in range(T):
            out.append(sorted((int(x["data_nbytes"][d]), int(x["data_get_nbytes"][d]), tuple(idx[ptr[d]:ptr[d + 1]]))
                              for d in x["dep_idx"][x["dep_ptr"][t]:x["dep_ptr"][t + 1]]))
        return out

    assert rows(p, hp, hi, None, None) == rows(q, q["holder_ptr"], q["holder_idx"], None, None)


def test_standin_plugin_problem_is_the_c4_problem():
    p = graphs.steal_problem(96, 4000, seed=3, replicas=3)
    ref = oracle.steal_balance(p)
    levels = np.asarray(ref["level"])
    keep = levels >= 0
    plugin, slot_task = plugin_from_problem(p, levels)
    q, rows, _ = plugin.rows.problem(plugin)
    q, rows = ordered_problem(q, rows)
    tasks = slot_task[rows]
    assert np.array_equal(tasks, np.flatnonzero(keep))  # the walk order is the problem's
    # the problem restricted to the tasks in a bin, with their levels as the bins' levels
    sub = dict(p, level_in=levels[keep])
    for k in ("victim", "duration", "fast"):
        sub[k] = np.asarray(p[k])[keep]
    cnt = np.diff(p["dep_ptr"])[keep]
    sub["dep_ptr"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    sub["dep_idx"] = np.concatenate([p["dep_idx"][p["dep_ptr"][t]:p["dep_ptr"][t + 1]] for t in np.flatnonzero(keep)])
    _same_problem(sub, q, int(keep.sum()))
    a = oracle.steal_balance(dict(p, level_in=levels))
    b = oracle.steal_balance(q)
    assert len(a["st_task"]) > 100
    assert np.array_equal(np.asarray(a["st_task"]), tasks[np.asarray(b["st_task"])])
    for k in ("st_victim", "st_thief", "st_level", "st_cost", "st_occ_victim", "st_occ_thief", "inflight_occ",
              "inflight_tasks", "idle_after", "sat_after", "checked"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
