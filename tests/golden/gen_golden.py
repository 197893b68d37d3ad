"""Golden-vector generator: replays the *reference* ``SchedulerState`` (imported
unmodified from ``/root/reference`` under the image's python3.9 + ``_refshim``)
over the synthetic graphs of ``distributed_amd/graphs.py`` and records every
placement it makes. Test infrastructure: it runs only in the build container,
and its outputs (``tests/golden/*.npz``) are the committed fixtures that pin the
oracle (``oracle/``) and, through it, the HIP engine.

Run (from the repo root)::

    PYTHONHASHSEED=0 /opt/conda/bin/python3.9 tests/golden/gen_golden.py [names...]

Replay protocol (SURVEY.md §8a "Replay/wave definition"):

* ``update_graph`` equivalent: TaskStates are created with ``SchedulerState.new_task``
  / ``TaskState.add_dependency`` (``distributed/scheduler.py:1821``, ``:1471``),
  sinks are wanted by one client, and every task is recommended ``"waiting"`` in
  descending priority (``:4600-4611``) through ``_transitions`` (``:2045``).
* round k completes, in ``run_id`` order, every task that was ``processing`` when
  the round started. Each completion is one stimulus exactly like
  ``Scheduler.handle_task_finished`` (``:5783-5797``): ``_transition(key, "memory",
  worker=..., nbytes=..., startstops=[compute start/stop])`` -> ``_transitions`` ->
  ``stimulus_queue_slots_maybe_opened`` (``:4983``).

Canonical tie-break (the reference leaves exact ties to set-iteration = hash order,
SURVEY.md §0): ``worker_objective`` gets the worker index appended as a last key
and ``idle_task_count`` / ``saturated`` iterate in ascending worker index. No
reference arithmetic is changed.

Recorded per placement (at ``_add_to_processing`` :3199, before it mutates):
task, worker, ``comm_bytes`` (the ``worker_objective`` sum, :3136-3138), the
objective's ``start_time`` (:3140-3141), ``ws.nbytes`` and the route taken
(0 non-rootish ``decide_worker``, 1 rootish+queuing, 2 rootish without queuing,
3 non-rootish no-dependency fast path). Recorded per round: per-worker occupancy,
nbytes, processing count, idle / saturated / idle_task_count membership and the
queue length.
"""
from __future__ import annotations

import importlib.util
import json
import math
import operator
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

if os.environ.get("PYTHONHASHSEED") != "0":
    # sets are iterated in hash order inside the reference; pin it
    env = dict(os.environ, PYTHONHASHSEED="0")
    sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))

import warnings  # noqa: E402

warnings.filterwarnings("ignore")
sys.path.insert(0, HERE)
import _refshim  # noqa: E402

_refshim.install()

import dask  # noqa: E402
import numpy as np  # noqa: E402

import distributed.scheduler  # noqa: E402,F401  (loads distributed.yaml defaults into dask.config)

_spec = importlib.util.spec_from_file_location("dgp_graphs", os.path.join(REPO, "distributed_amd", "graphs.py"))
graphs = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(graphs)

ROUTE_NONROOTISH, ROUTE_ROOTISH_Q, ROUTE_ROOTISH_NOQ, ROUTE_FASTPATH = 0, 1, 2, 3


def make_keys(g):
    """Reference keys whose key_split / key_split_group give the graph's prefixes/groups."""
    keys = []
    first = {}
    for t in range(g["n_tasks"]):
        gid = int(g["group_id"][t])
        gname = g["group_names"][gid]
        pname = g["prefix_names"][int(g["prefix_id"][t])]
        if gname == pname:
            keys.append(gname if gid not in first else (gname, t))
        else:
            keys.append((gname, t - first.setdefault(gid, t)))
        first.setdefault(gid, t)
    return keys


def build_state(g, cfg, addr_of=None):
    """Create the reference SchedulerState for graph ``g`` (no transitions yet). ``addr_of``:
    worker index -> address (default ``tcp://w{i:05d}:1``; any form whose order is the index
    order)."""
    addr_of = addr_of or (lambda i: f"tcp://w{i:05d}:1")
    from sortedcontainers import SortedDict

    from distributed.collections import HeapSet
    from distributed.core import Status
    from distributed.scheduler import ClientState, Scheduler, SchedulerState, WorkerState

    W = len(g["nthreads"])
    widx = {}

    class IdxSet(set):
        """set that iterates in ascending worker index (canonical tie-break)."""

        def __iter__(self):
            return iter(sorted(set.__iter__(self), key=lambda ws: widx[ws.address]))

    rec = {"task": [], "worker": [], "comm": [], "start": [], "wsnbytes": [], "route": []}
    tidx = {}

    class S(SchedulerState):
        _route = -1

        def transitions(self, recommendations, stimulus_id):
            self._transitions(recommendations, {}, {}, stimulus_id)

        stimulus_queue_slots_maybe_opened = Scheduler.stimulus_queue_slots_maybe_opened

        def log_event(self, *args, **kwargs):
            pass

        def worker_objective(self, ts, ws):
            return super().worker_objective(ts, ws) + (widx[ws.address],)

        def decide_worker_rootish_queuing_enabled(self):
            self._route = ROUTE_ROOTISH_Q
            return super().decide_worker_rootish_queuing_enabled()

        def decide_worker_rootish_queuing_disabled(self, ts):
            self._route = ROUTE_ROOTISH_NOQ
            return super().decide_worker_rootish_queuing_disabled(ts)

        def decide_worker_non_rootish(self, ts):
            vw = self.valid_workers(ts)
            if ts.dependencies or vw is not None or len(self.running) < len(self.workers):
                self._route = ROUTE_NONROOTISH
            else:
                self._route = ROUTE_FASTPATH
            return super().decide_worker_non_rootish(ts)

        def _add_to_processing(self, ts, ws, stimulus_id):
            comm = sum(d.get_nbytes() for d in ts.dependencies if ws not in (d.who_has or ()))
            start = ws.occupancy / ws.nthreads + comm / self.bandwidth
            rec["task"].append(tidx[ts.key])
            rec["worker"].append(widx[ws.address])
            rec["comm"].append(comm)
            rec["start"].append(start)
            rec["wsnbytes"].append(ws.nbytes)
            rec["route"].append(self._route)
            return super()._add_to_processing(ts, ws, stimulus_id=stimulus_id)

    s = S(
        aliases={}, clients={}, workers=SortedDict(), host_info={}, resources={}, tasks={},
        unrunnable=set(), queued=HeapSet(key=operator.attrgetter("priority")),
        validate=False, plugins=(),
    )
    s.idle_task_count = IdxSet()
    s.saturated = IdxSet()
    assert s.bandwidth == cfg["bandwidth"]
    for i in range(W):
        addr = addr_of(i)
        widx[addr] = i
        ws = WorkerState(address=addr, status=Status.running, pid=0, name=addr,
                         nthreads=int(g["nthreads"][i]), memory_limit=0, local_directory="",
                         nanny=None, server_id=addr, scheduler=s)
        s.workers[addr] = ws
        s.running.add(ws)
        s.aliases[addr] = addr
        s.total_nthreads += ws.nthreads
        s.check_idle_saturated(ws)

    keys = g["keys"] or make_keys(g)
    cs = ClientState("client-0")
    s.clients["client-0"] = cs
    run_spec = (operator.add, (), {})
    tss = []
    for t, key in enumerate(keys):
        ts = s.new_task(key, run_spec, "released")
        tidx[key] = t
        ts.priority = (0, 1, int(g["prio"][t]))
        ov = int(g["rootish_override"][t])
        if ov >= 0:
            ts._rootish = bool(ov)
        tss.append(ts)
        assert ts.prefix.name == g["prefix_names"][int(g["prefix_id"][t])], (key, ts.prefix.name)
        assert ts.group.name == g["group_names"][int(g["group_id"][t])], (key, ts.group.name)
    ptr, idx = g["dep_ptr"], g["dep_idx"]
    for t, ts in enumerate(tss):
        for d in idx[ptr[t]:ptr[t + 1]]:
            ts.add_dependency(tss[int(d)])
    if g.get("restr_flags") is not None:  # graphs.restrict: resolved valid workers
        rp, ri, rf = g["restr_ptr"], g["restr_idx"], g["restr_flags"]
        for t, ts in enumerate(tss):
            if rf[t] & 1:
                valid = {addr_of(int(w)) for w in ri[rp[t]:rp[t + 1]]}
                # a name no worker has: valid_workers drops it (:3059), so an otherwise
                # empty set is still a restriction, with no valid worker
                ts.worker_restrictions = valid | {"tcp://gone:1"}
                ts.loose_restrictions = bool(rf[t] & 2)
    for t, ts in enumerate(tss):
        if g["wanted"][t]:
            ts.who_wants = {cs}
            cs.wants_what.add(ts)
    for p, name in enumerate(g["prefix_names"]):
        if name in s.task_prefixes:
            assert s.task_prefixes[name].duration_average == g["prefix_default_dur"][p], name
    return s, tss, widx, rec, tidx


def snapshot(s, W, widx):
    occ = np.zeros(W)
    nb = np.zeros(W, np.int64)
    npr = np.zeros(W, np.int32)
    idle = np.zeros(W, np.uint8)
    sat = np.zeros(W, np.uint8)
    itc = np.zeros(W, np.uint8)
    for addr, ws in s.workers.items():
        i = widx[addr]
        occ[i] = ws.occupancy
        nb[i] = ws.nbytes
        npr[i] = len(ws.processing)
    for addr in s.idle:
        idle[widx[addr]] = 1
    for ws in s.saturated:
        sat[widx[ws.address]] = 1
    for ws in s.idle_task_count:
        itc[widx[ws.address]] = 1
    return occ, nb, npr, idle, sat, itc


STATE_CODES = {"released": 0, "waiting": 1, "processing": 2, "queued": 3, "no-worker": 4,
               "memory": 5, "erred": 6, "forgotten": 7}


def replay(g, cfg):
    """Run the reference replay; return (records dict, per-round arrays, seconds)."""
    s, tss, widx, rec, tidx = build_state(g, cfg)
    W = len(g["nthreads"])
    t0 = time.perf_counter()
    recs = {}
    for ts in sorted(tss, key=operator.attrgetter("priority"), reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    rounds = []
    nplaced = []
    stim = [len(rec["task"])]  # placements per stimulus: update_graph, then each completion
    done = 0
    while True:
        cur = len(rec["task"])
        batch = [tss[t] for t in rec["task"][done:cur]]
        snap = snapshot(s, W, widx)
        rounds.append(snap + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for ts in batch:
            assert ts.state == "processing", (ts.key, ts.state)
            t = ts.key
            i = tidx[t]
            sid = f"task-finished-{i}"
            r, cm, wm = s._transition(
                t, "memory", sid, worker=ts.processing_on.address, nbytes=int(g["nbytes"][i]),
                type=None, typename="int",
                startstops=[{"action": "compute", "start": float(g["start"][i]), "stop": float(g["stop"][i])}])
            n0 = len(rec["task"])
            s._transitions(r, cm, wm, sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
            stim.append(len(rec["task"]) - n0)
    secs = time.perf_counter() - t0
    states = np.array([STATE_CODES[ts.state] for ts in tss], np.uint8)
    rec["stim"] = stim
    return s, rec, rounds, nplaced, states, secs




def config_dict(saturation):
    return {
        "bandwidth": int(dask.config.get("distributed.scheduler.bandwidth")),
        "default_data_size": 1024,
        "unknown_duration": 0.5,
        "saturation": saturation,
    }


def save(name, g, cfg, rec, rounds, nplaced, states, secs):
    R = len(rounds)
    out = {k: g[k] for k in ("dep_ptr", "dep_idx", "prio", "prefix_id", "group_id", "wanted",
                             "rootish_override", "nbytes", "start", "stop", "nthreads",
                             "group_prefix", "prefix_default_dur")}
    out.update(
        pl_task=np.array(rec["task"], np.int32), pl_worker=np.array(rec["worker"], np.int32),
        pl_comm=np.array(rec["comm"], np.int64), pl_start=np.array(rec["start"], np.float64),
        pl_wsnbytes=np.array(rec["wsnbytes"], np.int64), pl_route=np.array(rec["route"], np.int8),
        round_nplaced=np.array(nplaced, np.int32),
        round_occ=np.stack([r[0] for r in rounds]), round_wnbytes=np.stack([r[1] for r in rounds]),
        round_nproc=np.stack([r[2] for r in rounds]), round_idle=np.stack([r[3] for r in rounds]),
        round_sat=np.stack([r[4] for r in rounds]), round_itc=np.stack([r[5] for r in rounds]),
        round_nqueued=np.array([r[6] for r in rounds], np.int32), final_state=states,
    )
    if g.get("restr_flags") is not None:
        out.update(restr_ptr=g["restr_ptr"], restr_idx=g["restr_idx"], restr_flags=g["restr_flags"])
    if "stim" in rec:  # placements made by each stimulus (update_graph, then every completion)
        out["stim_nplaced"] = np.array(rec["stim"], np.int32)
    sat = cfg["saturation"]
    meta = dict(name=name, prefix_names=list(g["prefix_names"]), group_names=list(g["group_names"]),
                config=dict(cfg, saturation=("inf" if math.isinf(sat) else sat)),
                reference_seconds=secs, n_placements=len(rec["task"]), n_rounds=R,
                generator="tests/golden/gen_golden.py", python=sys.version.split()[0],
                dask=dask.__version__)
    out["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(rec['task'])} placements, {R} rounds, reference {secs:.2f}s "
          f"-> {os.path.getsize(path) / 1e3:.0f} kB", flush=True)


def c1_dask_array_graph():
    """Config C1: dask.array ``(x + x.T).sum()`` on 10k x 10k with 1k chunks, materialised
    with the container's dask; priorities are this dask's ``dask.order`` (pinned as data)."""
    import dask.array as da
    from dask.core import get_dependencies
    from dask.order import order
    from dask.utils import key_split

    from distributed.utils import key_split_group

    x = da.random.RandomState(0).random_sample((10000, 10000), chunks=(1000, 1000))
    y = (x + x.T).sum()
    dsk = dict(y.__dask_graph__())
    o = order(dsk)
    keys = sorted(dsk, key=lambda k: o[k])
    kid = {k: i for i, k in enumerate(keys)}
    rows = [sorted(kid[d] for d in get_dependencies(dsk, k)) for k in keys]
    pnames, gnames, pid, gid, gpref = [], [], [], [], []
    for k in keys:
        p, gname = key_split(k), key_split_group(k)
        if p not in pnames:
            pnames.append(p)
        if gname not in gnames:
            gnames.append(gname)
            gpref.append(pnames.index(p))
        pid.append(pnames.index(p))
        gid.append(gnames.index(gname))
    ptr = np.zeros(len(keys) + 1, np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    idx = np.array([d for r in rows for d in r], np.int32)
    rng = np.random.default_rng(11)
    n = len(keys)
    # chunk outputs are 1000x1000 float64; reductions are scalars
    nbytes = np.array([8_000_000 if pnames[p] in ("random_sample", "transpose", "add") else 8 for p in pid],
                      np.int64)
    g = dict(name="c1_dask_array", dep_ptr=ptr, dep_idx=idx, prio=np.arange(n), prefix_id=pid,
             group_id=gid, prefix_names=pnames, group_names=gnames, group_prefix=gpref,
             prefix_default_dur=np.full(len(pnames), -1.0), nbytes=nbytes, start=np.zeros(n),
             stop=rng.uniform(0.01, 0.3, n), nthreads=np.full(4, 2), keys=keys)
    return graphs._finish(g)


def fixtures():
    inf = math.inf
    return {
        "c1_sat1.1": (c1_dask_array_graph, 1.1),
        "c1_satinf": (c1_dask_array_graph, inf),
        "c2mini_sat1.1": (lambda: graphs.random_dag(20000, 256, seed=0), 1.1),
        "c2mini_satinf": (lambda: graphs.random_dag(20000, 256, seed=0), inf),
        "c2var_sat1.1": (lambda: graphs.random_dag(6000, 64, seed=5, n_inner_prefixes=3, random_durations=True,
                                                   nthreads="random"), 1.1),
        "c2var_satinf": (lambda: graphs.random_dag(6000, 64, seed=6, n_inner_prefixes=3, random_durations=True,
                                                   nthreads="random"), inf),
        "c2var_sat2.5": (lambda: graphs.random_dag(4000, 32, seed=7, n_inner_prefixes=2, random_durations=True,
                                                   nthreads="random", root_frac=0.3), 2.5),
        # more task prefixes than the stream engine's descriptors carry (PD = 8): the
        # round-kernel engine's path
        "c2p12_sat1.1": (lambda: graphs.random_dag(3000, 64, seed=8, n_inner_prefixes=12, random_durations=True,
                                                   nthreads="random"), 1.1),
        "c2p12_satinf": (lambda: graphs.random_dag(2500, 48, seed=9, n_inner_prefixes=11, random_durations=True,
                                                   nthreads="random"), inf),
        "c3mini_sat1.1": (lambda: graphs.shuffle_graph(2000, 64, seed=2), 1.1),
        # decide_worker_non_rootish's no-dependency fast path at >= 20 and < 20 workers
        "nodep_w24_sat1.1": (lambda: no_dep_groups(24, 30, 12, 200, seed=21), 1.1),
        "nodep_w20_satinf": (lambda: no_dep_groups(20, 25, 9, 150, seed=22, nthreads="random"), inf),
        "nodep_w19_sat1.1": (lambda: no_dep_groups(19, 20, 10, 120, seed=23), 1.1),
        "c5mini_sat1.1": (lambda: graphs.map_tree_reduce(50000, 1024, seed=3), 1.1),
        "sat_factor_1.1": (lambda: root_only(10, [2, 1]), 1.1),
        "sat_factor_2.5": (lambda: root_only(10, [2, 1]), 2.5),
        "sat_factor_2.0": (lambda: root_only(10, [2, 1]), 2.0),
        "sat_factor_1.0": (lambda: root_only(10, [2, 1]), 1.0),
        "sat_factor_0.1": (lambda: root_only(10, [2, 1]), 0.1),
        "sat_factor_inf": (lambda: root_only(10, [2, 1]), inf),
        "occupancy_comm": (occupancy_comm_graph, 1.1),
        # worker restrictions / loose restrictions / no-worker (scheduler.py:3043-3107,
        # :8550-8593, :2761-2782): restricted roots leave the root-ish path (:2939)
        "restr_sat1.1": (lambda: graphs.restrict(graphs.random_dag(5000, 64, seed=51), 0.2, seed=52,
                                                 loose_frac=1.0), 1.1),
        "restr_satinf": (lambda: graphs.restrict(graphs.random_dag(4000, 48, seed=53, nthreads="random"), 0.25,
                                                 seed=54, max_valid=20, empty_frac=0.0, loose_frac=0.3), inf),
        "restr_nodep_w24": (lambda: graphs.restrict(no_dep_groups(24, 30, 12, 200, seed=55), 0.3, seed=56,
                                                    loose_frac=1.0), 1.1),
        # empty valid sets that are not loose: no-worker, and everything downstream waits
        "restr_noworker_sat1.1": (lambda: graphs.restrict(graphs.random_dag(5000, 64, seed=57), 0.2, seed=58),
                                  1.1),
    }


def no_dep_groups(n_workers, n_groups, group_size, n_agg, seed, nthreads=1):
    """The no-dependency fast path of ``decide_worker_non_rootish`` (scheduler.py:2283-2305):
    small groups of dependency-free tasks (``len(tg) <= 2 * total_nthreads``: not root-ish)
    placed by ``update_graph`` on ``idle or workers``; with >= 20 workers the pick is
    ``wp_vals[n_tasks % n]``, below 20 the least-occupied worker with a round-robin start.
    Aggregates over random loads follow."""
    rng = np.random.default_rng(seed)
    nl = n_groups * group_size
    n = nl + n_agg
    rows = [[] for _ in range(nl)] + [sorted(set(rng.integers(0, nl, 4).tolist())) for _ in range(n_agg)]
    ptr = np.zeros(n + 1, np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    gnames = [f"load-{k}" for k in range(n_groups)] + ["agg"]
    gid = [t // group_size for t in range(nl)] + [n_groups] * n_agg
    g = dict(name="nodep", dep_ptr=ptr, dep_idx=np.array([d for r in rows for d in r], np.int32),
             prio=rng.permutation(nl).tolist() + list(range(nl, n)), prefix_id=[0] * nl + [1] * n_agg,
             group_id=gid, prefix_names=["load", "agg"], group_names=gnames,
             group_prefix=[0] * n_groups + [1], prefix_default_dur=[-1.0, -1.0],
             nbytes=rng.lognormal(8, 2, n).astype(np.int64), start=np.zeros(n),
             stop=rng.uniform(0.001, 0.2, n),
             nthreads=(rng.integers(1, 3, n_workers) if nthreads == "random" else np.full(n_workers, nthreads)))
    return graphs._finish(g)


def root_only(n, nthreads):
    """``test_saturation_factor`` (distributed/tests/test_scheduler.py:637-683): 10 root
    tasks ``wait-i`` on workers with nthreads (2, 1)."""
    g = dict(name="roots", dep_ptr=np.zeros(n + 1, np.int64), dep_idx=np.zeros(0, np.int32),
             prio=np.arange(n), prefix_id=np.zeros(n), group_id=np.zeros(n), prefix_names=["wait"],
             group_names=["wait"], group_prefix=[0], prefix_default_dur=[-1.0],
             nbytes=np.full(n, 28), start=np.zeros(n), stop=np.full(n, 0.5), nthreads=nthreads,
             keys=[f"wait-{i}" for i in range(n)])
    return graphs._finish(g)


def occupancy_comm_graph():
    """``test_include_communication_in_occupancy`` (test_scheduler.py:1760-1799): x (2*bw
    bytes) and y (3*bw bytes) on different workers, z depends on both -> placed next to y,
    occupancy 0.5 s unknown compute + 2 s network = 2.5."""
    bw = 100_000_000
    g = dict(name="occ", dep_ptr=np.array([0, 0, 0, 2]), dep_idx=np.array([0, 1]), prio=np.arange(3),
             prefix_id=np.arange(3), group_id=np.arange(3), prefix_names=["mul", "mul2", "add_blocked"],
             group_names=["mul", "mul2", "add_blocked"], group_prefix=np.arange(3),
             prefix_default_dur=np.full(3, -1.0), nbytes=np.array([2 * bw, 3 * bw, 10]),
             start=np.zeros(3), stop=np.array([0.1, 0.1, 0.1]), nthreads=[1, 1],
             wanted=np.array([1, 1, 1]), keys=["mul", "mul2", "add_blocked"])
    return graphs._finish(g)


def main(names):
    fx = fixtures()
    for name in names or fx:
        mk, sat = fx[name]
        g = mk()
        graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = config_dict(sat)
        s, rec, rounds, nplaced, states, secs = replay(g, cfg)
        save(name, g, cfg, rec, rounds, nplaced, states, secs)


if __name__ == "__main__":
    main(sys.argv[1:])
