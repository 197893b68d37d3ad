"""Drives the drop-in ``GPUWorkStealing`` (distributed_amd/stealing.py) against the
reference ``WorkStealing`` (python3.9 + the reference; build container only, like
ext_driver.py). Called by ``tests/test_ext.py``.

Two identical scheduler states are built (tests/golden/gen_steal.build, canonical
tie-break instrumentation): one with the reference plugin, one with GPUWorkStealing
whose engine is a stand-in running the oracle restatement (oracle/steal.cpp, pinned
by the reference fixtures; the device kernels are checked against the same fixtures
on the GPU). Both balance() twice (the second call starts from the in-flight accounts
the first left). Checked equal: the ("request", log) events minus the wall-clock
field, both metrics, in_flight (victim, thief, durations), the steal-request messages
per victim, the stealable bins, idle / saturated / idle_task_count.
Prints one JSON line per case.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
if os.environ.get("PYTHONHASHSEED") != "0":
    import subprocess

    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, PYTHONHASHSEED="0")))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, REPO)

import gen_steal as GS  # noqa: E402  (shim + reference)

import numpy as np  # noqa: E402

from distributed_amd.stealing import GPUWorkStealing, ordered_problem, steal_problem_from_state  # noqa: E402
from oracle import oracle  # noqa: E402


class OracleEngine:
    def __init__(self):
        self.calls = 0

    def steal_balance(self, p):
        """The oracle on the problem in the device's walk order (dgp_steal_order's sort of
        the rows by (task_prio, task_arrival)); the outputs index the rows as given."""
        self.calls += 1
        if p.get("task_prio") is None:
            return oracle.steal_balance(p)
        perm = np.lexsort((p["task_arrival"], p["task_prio"]))
        q, _ = ordered_problem(p, perm)
        out = dict(oracle.steal_balance(q))
        out["st_task"] = perm[np.asarray(out["st_task"], np.int64)].astype(np.int32)
        if "level" in out:
            lv = np.empty_like(np.asarray(out["level"]))
            lv[perm] = out["level"]
            out["level"] = lv
        return out


def state_of(s, steal, events, comms):
    ev = [(topic, [tuple(e[1:]) for e in msg[1]]) for topic, msg in events if topic == "stealing"]
    return dict(
        events=ev,
        metrics={k: dict(v) for k, v in steal.metrics.items()},
        in_flight={ts.key: (i["victim"].address, i["thief"].address, i["victim_duration"], i["thief_duration"])
                   for ts, i in steal.in_flight.items()},
        in_flight_occ={ws.address: float(v) for ws, v in steal.in_flight_occupancy.items() if v},
        sent={a: [m["key"] for m in c.sent] for a, c in comms.items() if c.sent},
        stealable={a: [sorted(ts.key for ts in b) for b in bins] for a, bins in steal.stealable.items()},
        idle=sorted(s.idle), saturated=sorted(ws.address for ws in s.saturated),
        itc=sorted(ws.address for ws in s.idle_task_count),
    )


def rows_equal(steal):
    """The incremental task rows (StealRows) give the full rebuild's problem: identical
    columns, and per task the same dependencies (nbytes, get_nbytes, holders) up to their
    numbering."""
    a, ta, _ = steal_problem_from_state(steal)
    b, slots, _ = steal.problem()
    b, slots = ordered_problem(b, slots)  # the device's walk order
    tb = [steal.rows.task[int(i)] for i in slots]
    assert ta == tb, "task order"
    assert set(a) == set(b), (sorted(a), sorted(b))
    per_dep = ("dep_idx", "data_nbytes", "data_get_nbytes", "holder_ptr", "holder_idx")
    for k in a:
        if k in per_dep:
            continue
        if isinstance(a[k], np.ndarray):
            assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k

    def deps(p):
        out = []
        for t in range(len(p["dep_ptr"]) - 1):
            r = []
            for d in p["dep_idx"][p["dep_ptr"][t]:p["dep_ptr"][t + 1]]:
                h = tuple(p["holder_idx"][p["holder_ptr"][d]:p["holder_ptr"][d + 1]])
                r.append((int(p["data_nbytes"][d]), int(p["data_get_nbytes"][d]), h))
            out.append(sorted(r))
        return out

    assert deps(a) == deps(b), "dependency rows"
    for p in (a, b):  # rows ascending (the device's dependency walks assume it)
        for t in range(len(p["dep_ptr"]) - 1):
            r = p["dep_idx"][p["dep_ptr"][t]:p["dep_ptr"][t + 1]]
            assert np.all(np.diff(r) > 0), "row order"


def run(name, case):
    out = {}
    for kind in ("reference", "gpu"):
        kw = {}
        if kind == "gpu":
            eng = OracleEngine()
            kw = dict(steal_base=GPUWorkStealing, steal_kwargs=dict(engine_factory=lambda: eng, validate=True))
        s, steal, widx, tidx, data, work, deps_of, events, comms = GS.build(**case, **kw)
        for _ in range(2):
            if kind == "gpu":
                rows_equal(steal)
            steal.balance()
        out[kind] = state_of(s, steal, events, comms)
        if kind == "gpu":
            rebuilt = steal.gpu_stats["rows_rebuilt"]
    ref, gpu = out["reference"], out["gpu"]
    diff = [k for k in ref if ref[k] != gpu[k]]
    n_req = sum(len(e[1]) for e in ref["events"])
    return dict(case=name, requests=n_req, balance_events=len(ref["events"]), differ=diff, rows_rebuilt=rebuilt)


CASES = {
    "c4mini": dict(W=256, T=5000, nthreads=2, hot_frac=0.1, seed=1),
    "many_saturated": dict(W=320, T=6000, nthreads=2, hot_frac=0.1, seed=3, dist="uniform"),
    "restricted": dict(W=256, T=5000, nthreads=2, hot_frac=0.1, seed=11, restrict=0.3),
    "spread": dict(W=64, T=224, nthreads=2, hot_frac=0.25, seed=5, dist="uniform", nprefix=2, nb_mu=8.0),
}

if __name__ == "__main__":
    import warnings

    warnings.filterwarnings("ignore")
    for nm in sys.argv[1:] or CASES:
        print(json.dumps(run(nm, CASES[nm])), flush=True)
