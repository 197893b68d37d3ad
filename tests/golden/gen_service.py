"""Golden vectors for the service-mode boundary (``dgp_tasks_finished``): the reference's
own ``Scheduler.stimulus_task_finished`` (``distributed/scheduler.py:5025-5092``) answers a
stream of task-finished messages that mixes the genuine completions of the replay protocol
(``gen_golden.py``) with the stale, duplicate and already-in-memory reports a live
scheduler receives. Test infrastructure: runs only in the build container
(python3.9 + ``_refshim``), like ``gen_golden.py``.

Run (from the repo root)::

    PYTHONHASHSEED=0 /opt/conda/bin/python3.9 tests/golden/gen_service.py

Per message the fixture stores what the caller sends (task, worker, run_id = placement-log
position of the compute-task it answers, nbytes, compute start/stop) and the reference's
answer, classified as in ``include/dgplace.h`` ``DGP_TF_*``:

* ``ACCEPTED``   ``_transition(key, "memory")`` ran (:5090)
* ``FREE_KEYS``  the returned worker messages hold ``free-keys`` (:5036-5079)
* ``ADD_KEYS``   ``Scheduler.add_keys`` was called (:5082-5083)
* ``RELEASE``    the returned recommendations are ``{key: "released"}`` (:5080-5081); this
  generator does not apply them, the engine leaves them to its caller as well
* ``UNKNOWN_WORKER`` the worker is not in ``Scheduler.workers``: ``handle_task_finished``
  returns before the stimulus (:5786-5787)

Injected messages never change scheduler state (same-worker duplicates are idempotent in
``WorkerState.add_replica`` :829-830), so the placement log and the per-round snapshots
equal those of the plain replay; both are stored and checked.

With ``p_steal`` (the ``svc_steal_*`` fixtures) confirmed steals are interleaved too:
before a message, a processing task moves to another worker exactly as
``WorkStealing.move_task_confirm``'s "confirm" branch does it (distributed/stealing.py
:376-384 and the finally clause :396-399: remove_from_processing on the victim,
add_to_processing on the thief, a new compute-task via ``send_task_to_worker``,
check_idle_saturated of thief and victim). The steals change the later placements; the
fixture stores them (``steal_msg`` = index of the message they precede, ``steal_task``,
``steal_thief``) with the placement log and snapshots they lead to.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if os.environ.get("PYTHONHASHSEED") != "0":
    import subprocess

    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, PYTHONHASHSEED="0")))
sys.path.insert(0, HERE)

import gen_golden as G  # noqa: E402  (installs the shim, imports the reference)

import math  # noqa: E402
import operator  # noqa: E402

import dask  # noqa: E402
import numpy as np  # noqa: E402

ACCEPTED, FREE_KEYS, ADD_KEYS, RELEASE, UNKNOWN_WORKER = 0, 1, 2, 3, 4


def replay_service(g, cfg, seed, p_inject=0.35, p_steal=0.0):
    from distributed.scheduler import Scheduler

    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    W = len(g["nthreads"])
    N = g["n_tasks"]
    addr = {i: a for a, i in widx.items()}
    rng = np.random.default_rng(seed)
    called = {"add_keys": 0}

    def add_keys(self, worker, keys=(), stimulus_id=None):  # Scheduler.add_keys, no comms
        called["add_keys"] += 1
        ws = self.workers[worker]
        for key in keys:
            ts = self.tasks.get(key)
            if ts is not None and ts.state == "memory":
                self.add_replica(ts, ws)
        return "OK"

    type(s).add_keys = add_keys
    type(s).stimulus_task_finished = Scheduler.stimulus_task_finished
    run0 = None  # the reference's run_id counter value of placement 0

    recs = {}
    for ts in sorted(tss, key=lambda t: t.priority, reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    run0 = tss[rec["task"][0]].run_id
    msgs = {k: [] for k in ("task", "worker", "run_id", "nbytes", "start", "stop", "status")}
    round_ptr = [0]
    rounds, nplaced = [], []
    done = 0
    completed = []  # tasks accepted so far (duplicates are drawn from these)
    ran_on = {}     # task -> the worker its accepted completion came from

    steals = {"msg": [], "task": [], "thief": []}
    stolen = set()

    def steal():
        """WorkStealing.move_task_confirm, confirm branch (stealing.py:376-384, :396-399)."""
        proc = [ts for ts in s.tasks.values() if ts.state == "processing"]
        if not proc or W < 2:
            return
        ts = proc[int(rng.integers(0, len(proc)))]
        victim = ts.processing_on
        h = (widx[victim.address] + 1 + int(rng.integers(0, W - 1))) % W
        thief = s.workers[addr[h]]
        ts.processing_on = thief
        victim.remove_from_processing(ts)
        thief.add_to_processing(ts)
        s._task_to_msg(ts)  # send_task_to_worker: the thief's compute-task, a new run_id
        s.check_idle_saturated(thief)
        s.check_idle_saturated(victim)
        steals["msg"].append(len(msgs["task"]))
        steals["task"].append(tidx[ts.key])
        steals["thief"].append(h)
        stolen.add(tidx[ts.key])

    def send(t, w, run_id, nbytes, start, stop, ref_run=None):
        """One task-finished message through the reference; returns its class."""
        msgs["task"].append(t)
        msgs["worker"].append(w)
        msgs["run_id"].append(run_id)
        msgs["nbytes"].append(nbytes)
        msgs["start"].append(start)
        msgs["stop"].append(stop)
        if w >= W:
            st = UNKNOWN_WORKER
        else:
            key = tss[t].key if t < N else ("forgotten", t)
            ts = s.tasks.get(key)
            before = ts.state if ts is not None else None
            sid = f"task-finished-{len(msgs['task'])}"
            k0 = called["add_keys"]
            r, cm, wm = s.stimulus_task_finished(
                key, addr[w], sid, run_id + run0 if ref_run is None else ref_run, nbytes=nbytes, type=None, typename="int", metadata=None,
                startstops=[{"action": "compute", "start": start, "stop": stop}])
            if called["add_keys"] > k0:
                st = ADD_KEYS
            elif any(m.get("op") == "free-keys" for v in wm.values() for m in v):
                st = FREE_KEYS
            elif r == {key: "released"} and before == "processing" and ts.state == "processing":
                st = RELEASE  # not applied (the engine leaves it to the caller)
            else:
                assert before == "processing" and ts.state != "processing", (key, before, ts.state, r, wm)
                st = ACCEPTED
                s._transitions(r, cm, wm, sid)
                s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
                completed.append(t)
        msgs["status"].append(st)
        return st

    while True:
        cur = len(rec["task"])
        batch = list(range(done, cur))
        rounds.append(G.snapshot(s, W, widx) + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for pos in batch:
            while p_steal and rng.random() < p_steal:
                steal()
            while rng.random() < p_inject:  # crafted messages before the genuine one
                kind = int(rng.integers(0, 6))
                proc = [ts for ts in s.tasks.values() if ts.state == "processing" and tidx[ts.key] not in stolen]
                if kind == 0 and completed:  # duplicate of an accepted completion, same worker
                    t = completed[int(rng.integers(0, len(completed)))]
                    ts = tss[t]
                    w = ran_on[t]  # the worker that ran it
                    send(t, w, int(rec["task"].index(t)), 77, 0.0, 0.5, ref_run=int(ts.run_id))
                elif kind == 1 and proc:  # stale run of a processing task, from another worker
                    ts = proc[int(rng.integers(0, len(proc)))]
                    w = (widx[ts.processing_on.address] + 1 + int(rng.integers(0, W - 1))) % W
                    send(tidx[ts.key], w, rec["task"].index(tidx[ts.key]) - 1, 5, 0.0, 0.5, ref_run=int(ts.run_id) - 1)
                elif kind == 2 and s.queued:  # a queued task
                    ts = s.queued.peek()
                    send(tidx[ts.key], int(rng.integers(0, W)), 0, 5, 0.0, 0.5)
                elif kind == 3:  # a key the scheduler does not know (forgotten)
                    send(N + int(rng.integers(0, 100)), int(rng.integers(0, W)), 0, 5, 0.0, 0.5)
                elif kind == 4:  # a worker that is not registered
                    send(int(rng.integers(0, N)), W + int(rng.integers(0, 5)), 0, 5, 0.0, 0.5)
                elif kind == 5 and proc:  # stale run_id from the worker it is processing on
                    ts = proc[int(rng.integers(0, len(proc)))]
                    send(tidx[ts.key], widx[ts.processing_on.address], rec["task"].index(tidx[ts.key]) - 1, 5, 0.0, 0.5,
                         ref_run=int(ts.run_id) - 1)
            t = rec["task"][pos]
            ts = tss[t]
            assert ts.state == "processing", (ts.key, ts.state)
            ran_on[t] = widx[ts.processing_on.address]
            st = send(t, ran_on[t], pos, int(g["nbytes"][t]), float(g["start"][t]), float(g["stop"][t]),
                      ref_run=int(ts.run_id))
            assert st == ACCEPTED
        round_ptr.append(len(msgs["task"]))
    states = np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8)
    return rec, rounds, nplaced, states, msgs, round_ptr, steals


def replay_add_workers(g, cfg, seed, n_add, max_nthreads=4, interleave=False, n_paused=0):
    """The replay protocol's completions as task-finished messages, with ``n_add`` workers
    joining at random points of the first half of the stream, exactly as
    ``Scheduler.add_worker`` (distributed/scheduler.py:4308-4441) changes the placement
    state: the WorkerState enters ``workers`` (a SortedDict by address, :3746, :4353) /
    ``running``, ``total_nthreads`` grows (:4383), ``check_idle_saturated(ws)`` (:4398), then
    ``bulk_schedule_unrunnable_after_adding_worker`` and ``stimulus_queue_slots_maybe_opened``
    (:4416-4420). Addresses sort after the existing ones (the new worker's index is the next
    one), or with ``interleave`` anywhere among them: the canonical worker index is always
    the SortedDict rank, so every later worker's index moves up by one at such a join.
    ``n_paused`` of the joining workers join paused (status paused: not running, no refill,
    :4368-4369, :4416) and resume later through ``Scheduler.handle_worker_status_change``
    (:5850-5883). Stored: ``add_msg`` (the message index each addition precedes),
    ``add_nthreads``, ``add_pos`` (its index at the join), ``add_running``; ``res_msg`` /
    ``res_worker`` (the resumes: message index, the worker's index then); messages, placements
    and snapshots carry the index of their time; snapshots are as wide as the final worker
    count (0 for workers not yet added)."""
    from distributed.core import Status
    from distributed.scheduler import Scheduler, WorkerState

    addr_of = (lambda i: f"tcp://w{100 * i:07d}:1") if interleave else None
    s, tss, widx, rec, tidx = G.build_state(g, cfg, addr_of)
    W0 = len(g["nthreads"])
    W = W0 + n_add
    N = g["n_tasks"]
    rng = np.random.default_rng(seed)
    type(s).stimulus_task_finished = Scheduler.stimulus_task_finished
    type(s).handle_worker_status_change = Scheduler.handle_worker_status_change
    type(s).send_all = lambda self, client_msgs, worker_msgs: None
    s.extensions = {}
    add_at = sorted(int(x) for x in rng.choice(N // 2, n_add, replace=False))
    add_nt = [int(x) for x in rng.integers(1, max_nthreads + 1, n_add)]
    add_near = [int(x) for x in rng.integers(0, W0, n_add)]  # interleave: the address follows worker j's
    paused_k = set(int(x) for x in rng.choice(n_add, n_paused, replace=False)) if n_paused else set()
    added = {"msg": [], "nthreads": [], "pos": [], "running": [], "addr": []}
    resumes = {"msg": [], "worker": []}
    res_at = {}  # message index -> address to resume

    def add_worker(k, nthreads):
        addr = f"tcp://w{100 * add_near[k] + 1 + k:07d}:1" if interleave else f"tcp://w{W0 + k:05d}:1"
        running = k not in paused_k
        ws = WorkerState(address=addr, status=Status.running if running else Status.paused, pid=0, name=addr,
                         nthreads=nthreads, memory_limit=0, local_directory="", nanny=None, server_id=addr,
                         scheduler=s)
        s.workers[addr] = ws
        for i, a in enumerate(s.workers):  # the SortedDict rank is the canonical index
            widx[a] = i
        if running:
            s.running.add(ws)
        s.aliases[addr] = addr
        s.total_nthreads += nthreads
        s.check_idle_saturated(ws)
        sid = f"add-worker-{k}"
        if running:
            s.transitions(s.bulk_schedule_unrunnable_after_adding_worker(ws), sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
        else:  # resumes somewhere in the rest of the stream
            res_at.setdefault(int(rng.integers(len(msgs["task"]) + 1, N)), []).append(addr)
        added["addr"].append(addr)
        return widx[addr], running

    recs = {}
    for ts in sorted(tss, key=lambda t: t.priority, reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    stim = [len(rec["task"])]  # placements per event: update_graph, then each join / completion
    msgs = {k: [] for k in ("task", "worker", "run_id", "nbytes", "start", "stop", "status")}
    round_ptr = [0]
    rounds, nplaced = [], []
    done = 0
    k_add = 0
    while True:
        cur = len(rec["task"])
        batch = list(range(done, cur))
        rounds.append(G.snapshot(s, W, widx) + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for pos in batch:
            while k_add < n_add and add_at[k_add] <= len(msgs["task"]):
                added["msg"].append(len(msgs["task"]))
                added["nthreads"].append(add_nt[k_add])
                n0 = len(rec["task"])
                p, running = add_worker(k_add, add_nt[k_add])
                added["pos"].append(p)
                added["running"].append(int(running))
                stim.append(len(rec["task"]) - n0)
                k_add += 1
            for a in res_at.pop(len(msgs["task"]), ()):
                resumes["msg"].append(len(msgs["task"]))
                resumes["worker"].append(widx[a])
                n0 = len(rec["task"])
                s.handle_worker_status_change("running", a, f"resume-{a}")
                stim.append(len(rec["task"]) - n0)
            t = rec["task"][pos]
            ts = tss[t]
            assert ts.state == "processing", (ts.key, ts.state)
            w = widx[ts.processing_on.address]
            sid = f"task-finished-{len(msgs['task'])}"
            r, cm, wm = s.stimulus_task_finished(
                ts.key, ts.processing_on.address, sid, int(ts.run_id), nbytes=int(g["nbytes"][t]), type=None,
                typename="int", metadata=None,
                startstops=[{"action": "compute", "start": float(g["start"][t]), "stop": float(g["stop"][t])}])
            assert ts.state != "processing"
            n0 = len(rec["task"])
            s._transitions(r, cm, wm, sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
            stim.append(len(rec["task"]) - n0)
            for k, v in zip(("task", "worker", "run_id", "nbytes", "start", "stop", "status"),
                            (t, w, pos, int(g["nbytes"][t]), float(g["start"][t]), float(g["stop"][t]), ACCEPTED)):
                msgs[k].append(v)
        round_ptr.append(len(msgs["task"]))
    assert k_add == n_add, (k_add, n_add)
    assert not res_at or min(res_at) >= len(msgs["task"]), res_at  # resumes past the stream's end are dropped
    rec["stim"] = stim
    states = np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8)
    added["resumes"] = resumes
    return rec, rounds, nplaced, states, msgs, round_ptr, added


def main_add_workers(only):
    cases = {
        # 48 workers x 1-4 threads, root group of 400 tasks: root-ish (400 > 2 * total_nthreads)
        # at the start, queued roots left when the workers join
        "svcaddw_c2var_sat1.1": (lambda: G.graphs.random_dag(4000, 48, seed=21, n_inner_prefixes=3,
                                                              random_durations=True, nthreads="random"), 1.1, 5, 24),
        "svcaddw_c2mini_satinf": (lambda: G.graphs.random_dag(3000, 32, seed=22), float("inf"), 6, 12),
        "svcaddw_c2mini_sat1.0": (lambda: G.graphs.random_dag(3000, 60, seed=23), 1.0, 7, 70),
        # 1,000 workers (worker state in LDS) growing to 1,300: the stream engine switches to
        # its global-memory worker layout part-way through the stream
        "svcaddw_w1000_sat1.1": (lambda: G.graphs.random_dag(30000, 1000, seed=24), 1.1, 8, 300),
        # worker restrictions (30 % of the tasks, half of them loose) and 16 task prefixes:
        # the stream engine's restricted decisions and its 16-prefix dicts across joins
        "svcaddw_restr_sat1.1": (lambda: G.graphs.restrict(G.graphs.random_dag(3000, 48, seed=25, n_inner_prefixes=3,
                                                                                random_durations=True,
                                                                                nthreads="random"),
                                                            0.3, seed=25, empty_frac=0.0), 1.1, 9, 24),
        "svcaddw_p16_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=26, n_inner_prefixes=15,
                                                            random_durations=True, nthreads="random"), 1.1, 10, 24),
        # addresses that sort among the known ones (a real cluster's tcp://host:<port>): every
        # later worker's canonical index moves up at each join; 4 of them join paused and
        # resume later
        "svcaddw_order_sat1.1": (lambda: G.graphs.random_dag(4000, 40, seed=27, n_inner_prefixes=3,
                                                              random_durations=True, nthreads="random"), 1.1, 11, 24,
                                 dict(interleave=True, n_paused=4)),
        "svcaddw_order_satinf": (lambda: G.graphs.random_dag(3000, 32, seed=28), float("inf"), 12, 16,
                                 dict(interleave=True, n_paused=3)),
    }
    for name, (mk, sat, seed, n_add, *kw) in cases.items():
        if only and name not in only:
            continue
        g = mk()
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        rec, rounds, nplaced, states, msgs, round_ptr, added = replay_add_workers(g, cfg, seed, n_add,
                                                                                 **(kw[0] if kw else {}))
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(msg_task=np.array(msgs["task"], np.int32), msg_worker=np.array(msgs["worker"], np.int32),
                 msg_runid=np.array(msgs["run_id"], np.int64), msg_nbytes=np.array(msgs["nbytes"], np.int64),
                 msg_start=np.array(msgs["start"]), msg_stop=np.array(msgs["stop"]),
                 msg_status=np.array(msgs["status"], np.int8), msg_round_ptr=np.array(round_ptr, np.int64),
                 add_msg=np.array(added["msg"], np.int64), add_nthreads=np.array(added["nthreads"], np.int32),
                 add_pos=np.array(added["pos"], np.int32), add_running=np.array(added["running"], np.int8),
                 res_msg=np.array(added["resumes"]["msg"], np.int64),
                 res_worker=np.array(added["resumes"]["worker"], np.int32),
                 add_addr=np.array(added["addr"], dtype="U32"),
                 addr_step=np.array(100 if (kw and kw[0].get("interleave")) else 0, np.int32))
        np.savez_compressed(path, **z)
        routes = np.bincount(np.array(rec["route"]), minlength=4).tolist()
        print(f"{name}: {len(msgs['task'])} messages, {len(added['msg'])} workers added, routes {routes}")


TOKEN2 = "f9e8d7c6b5a49382716051e4d3c2b1a0"


def replay_second_graph(g, g2, cfg, seed, at_frac, n_add=0, dep_frac=0.0, restr=False, user_prio=0, recompute=False):
    """The replay protocol's completions as task-finished messages, with a second,
    independent graph ``g2`` submitted part-way through, the way
    ``Scheduler._create_taskstate_from_graph`` (distributed/scheduler.py:4512-4653) adds it:
    new TaskStates (keys of their own groups ``<prefix>-TOKEN2``: the prefixes are the first
    graph's, so each TaskPrefix keeps its duration average), priority ``(0, 2, i)`` (a later
    generation than the first graph's ``(0, 1, i)``), dependencies, ``who_wants``, then every
    new task recommended "waiting" in priority order. The new tasks get indices N.. in the
    fixture; their completions follow the protocol like the others'.

    ``dep_frac``: that fraction of the new tasks also depends on one earlier task (in memory,
    processing, waiting or queued when the graph arrives); the scheduler's state after the
    submission is dumped as resync rows (the engine appends the graph, the scheduler decides
    that stimulus, the engine resyncs).

    ``restr``: ``g2`` carries worker restrictions (graphs.restrict rows, set on the new
    TaskStates as build_state does): the scheduler's state after the submission is dumped as
    resync rows too (the engine appends the graph deferred, the scheduler decides that
    stimulus, the engine resyncs and takes the rows, dgp_update_restrictions).

    ``user_prio``: the later graph is submitted with that user priority (``_set_priorities``
    :4934-4981 puts ``-priority`` first in the tuple), so its tasks outrank every earlier one:
    the resync rows are dumped after the submission and the fixture holds every task's rank
    in the merged order (``g2_prio_all``, the engine's re-rank: dgp_set_priorities)."""
    from distributed.core import Status
    from distributed.scheduler import Scheduler, WorkerState

    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    W0 = len(g["nthreads"])
    W = W0 + n_add
    N = g["n_tasks"]
    type(s).stimulus_task_finished = Scheduler.stimulus_task_finished
    recs = {}
    for ts in sorted(tss, key=lambda t: t.priority, reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    add_at = int(at_frac * N)
    # workers joining (with n_add: Scheduler.add_worker's placement part, as in replay_add_workers)
    rng = np.random.default_rng(seed)
    join_at = sorted(int(x) for x in rng.choice(N, n_add, replace=False)) if n_add else []
    join_nt = [int(x) for x in rng.integers(1, 5, n_add)]
    joins = {"msg": [], "nthreads": []}

    def join(i, nthreads):
        addr = f"tcp://w{i:05d}:1"
        widx[addr] = i
        ws = WorkerState(address=addr, status=Status.running, pid=0, name=addr, nthreads=nthreads, memory_limit=0,
                         local_directory="", nanny=None, server_id=addr, scheduler=s)
        s.workers[addr] = ws
        s.running.add(ws)
        s.aliases[addr] = addr
        s.total_nthreads += nthreads
        s.check_idle_saturated(ws)
        s.transitions(s.bulk_schedule_unrunnable_after_adding_worker(ws), f"add-worker-{i}")
        s.stimulus_queue_slots_maybe_opened(stimulus_id=f"add-worker-{i}")
    nb = list(g["nbytes"]) + list(g2["nbytes"])
    a0 = list(g["start"]) + list(g2["start"])
    b0 = list(g["stop"]) + list(g2["stop"])
    cs = s.clients["client-0"]
    run_spec = (operator.add, (), {})
    added = {"msg": -1}
    ext = {"ptr": None, "idx": None, "dumps": [], "nplaced": 0}
    rng_dep = np.random.default_rng(seed + 7)

    def submit():
        keys2 = G.make_keys(g2)
        new = []
        for t, key in enumerate(keys2):
            ts = s.new_task(key, run_spec, "released")
            tidx[key] = N + t
            ts.priority = (-user_prio, 2, int(g2["prio"][t]))
            ov = int(g2["rootish_override"][t])
            if ov >= 0:
                ts._rootish = bool(ov)
            new.append(ts)
        ptr, idx = g2["dep_ptr"], g2["dep_idx"]
        live = ("memory", "processing", "waiting", "queued") + (("released",) if recompute else ())
        earlier = [ts for ts in tss if ts.state in live]
        rows = []
        for t, ts in enumerate(new):
            row = [int(d) for d in idx[ptr[t]:ptr[t + 1]]]
            for d in row:
                ts.add_dependency(new[d])
            if dep_frac and earlier and rng_dep.random() < dep_frac:
                o = earlier[int(rng_dep.integers(0, len(earlier)))]
                ts.add_dependency(o)
                row.append(-1 - tidx[o.key])
            rows.append(row)
            if g2["wanted"][t]:
                ts.who_wants = {cs}
                cs.wants_what.add(ts)
            if restr and g2["restr_flags"][t] & 1:  # as build_state sets a fixture graph's
                rp, ri = g2["restr_ptr"], g2["restr_idx"]
                ts.worker_restrictions = {f"tcp://w{int(w):05d}:1" for w in ri[rp[t]:rp[t + 1]]} | {"tcp://gone:1"}
                ts.loose_restrictions = bool(g2["restr_flags"][t] & 2)
        ext["ptr"] = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
        ext["idx"] = np.array([d for r in rows for d in r], np.int32)
        recs2 = {ts.key: "waiting" for ts in sorted(new, key=lambda t: t.priority, reverse=True)}
        if recompute:  # the set orders the recompute follows (distributed_amd/loss.py, as the extension passes them)
            LS = _load_repo_module("loss")
            chain = LS.graph_cascade(new)
            assert chain, "no released earlier dependency"
            rows = LS.graph_orders(new, chain, lambda ts: tidx[ts.key])
            ext["lo_task"] = np.array([r[0] for r in rows], np.int32)
            ext["lo_kind"] = np.array([r[1] for r in rows], np.int8)
            ext["lo_rowptr"] = np.concatenate([[0], np.cumsum([len(r[2]) for r in rows])]).astype(np.int64)
            ext["lo_idx"] = np.array([x for r in rows for x in r[2]], np.int32)
            ext["n_recomputed"] = len(chain)
        s._transitions(recs2, {}, {}, "update-graph-2")
        if dep_frac or restr or user_prio:
            gall = dict(prefix_names=g["prefix_names"], prefix_default_dur=g["prefix_default_dur"],
                        group_names=list(g["group_names"]) + list(g2["group_names"]))
            ext["dumps"].append(_dump(s, gall, tidx, widx, [ts.key for ts in tss] + [ts.key for ts in new]))
        tss.extend(new)
        ext["prio_all"] = np.empty(len(tss), np.int64)
        ext["prio_all"][sorted(range(len(tss)), key=lambda t: tss[t].priority)] = np.arange(len(tss))

    msgs = {k: [] for k in ("task", "worker", "run_id", "nbytes", "start", "stop", "status")}
    stim = [len(rec["task"])]
    round_ptr = [0]
    rounds, nplaced = [], []
    done = 0
    while True:
        cur = len(rec["task"])
        batch = list(range(done, cur))
        rounds.append(G.snapshot(s, W, widx) + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for pos in batch:
            while len(joins["msg"]) < n_add and join_at[len(joins["msg"])] <= len(msgs["task"]):
                k = len(joins["msg"])
                joins["msg"].append(len(msgs["task"]))
                joins["nthreads"].append(join_nt[k])
                n0 = len(rec["task"])
                join(W0 + k, join_nt[k])
                stim.append(len(rec["task"]) - n0)
            if added["msg"] < 0 and len(msgs["task"]) >= add_at:
                added["msg"] = len(msgs["task"])
                n0 = len(rec["task"])
                submit()
                stim.append(len(rec["task"]) - n0)
                ext["nplaced"] = stim[-1]
            t = rec["task"][pos]
            ts = tss[t]
            assert ts.state == "processing", (ts.key, ts.state)
            w = widx[ts.processing_on.address]
            sid = f"task-finished-{len(msgs['task'])}"
            r, cm, wm = s.stimulus_task_finished(
                ts.key, ts.processing_on.address, sid, int(ts.run_id), nbytes=int(nb[t]), type=None,
                typename="int", metadata=None,
                startstops=[{"action": "compute", "start": float(a0[t]), "stop": float(b0[t])}])
            assert ts.state != "processing"
            n0 = len(rec["task"])
            s._transitions(r, cm, wm, sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
            stim.append(len(rec["task"]) - n0)
            for k, v in zip(("task", "worker", "run_id", "nbytes", "start", "stop", "status"),
                            (t, w, pos, int(nb[t]), float(a0[t]), float(b0[t]), ACCEPTED)):
                msgs[k].append(v)
        round_ptr.append(len(msgs["task"]))
    assert added["msg"] >= 0 and len(joins["msg"]) == n_add
    rec["stim"] = stim
    states = np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8)
    return rec, rounds, nplaced, states, msgs, round_ptr, added["msg"], joins, ext


def main_second_graph(only):
    cases = {
        "svcgraph_c2var_sat1.1": (dict(n=3000, w=32, seed=31, n_inner_prefixes=3, random_durations=True,
                                       nthreads="random"), dict(n=2000, seed=32), 1.1, 0.3),
        "svcgraph_c2mini_satinf": (dict(n=2500, w=24, seed=33), dict(n=1500, seed=34), float("inf"), 0.5, 0),
        # the second graph and 40 workers joining in one stream
        "svcgraph_joins_sat1.1": (dict(n=4000, w=40, seed=35, n_inner_prefixes=2, random_durations=True,
                                       nthreads="random"), dict(n=3000, seed=36), 1.1, 0.4, 40),
        # restrictions on the first graph (the later one has none) and 12 task prefixes
        "svcgraph_restr_sat1.1": (dict(n=3000, w=32, seed=37, n_inner_prefixes=11, random_durations=True,
                                       nthreads="random", restrict=0.3), dict(n=2000, seed=38), 1.1, 0.3, 8),
        # later graphs that depend on earlier tasks (the scheduler decides their stimulus, then resync)
        "svcgdep_c2var_sat1.1": (dict(n=3000, w=32, seed=41, n_inner_prefixes=3, random_durations=True,
                                      nthreads="random"), dict(n=2000, seed=42), 1.1, 0.3, 0, 0.2),
        "svcgdep_c2mini_satinf": (dict(n=2500, w=24, seed=43), dict(n=1500, seed=44), float("inf"), 0.5, 0, 0.3),
        "svcgdep_joins_sat1.0": (dict(n=3000, w=32, seed=45, n_inner_prefixes=2, random_durations=True,
                                      nthreads="random"), dict(n=2000, seed=46), 1.0, 0.4, 12, 0.1),
        # later graphs with worker restrictions (deferred append, the scheduler's stimulus, resync + rows)
        "svcgrst_c2var_sat1.1": (dict(n=3000, w=32, seed=47, n_inner_prefixes=3, random_durations=True,
                                      nthreads="random"), dict(n=2000, seed=48, restrict=0.3), 1.1, 0.3, 0, 0.0),
        "svcgrst_dep_satinf": (dict(n=2500, w=24, seed=49), dict(n=1500, seed=50, restrict=0.2), float("inf"), 0.5, 0,
                               0.2),
        # later graphs submitted with a user priority: they outrank the earlier tasks (re-rank)
        "svcgprio_c2var_sat1.1": (dict(n=3000, w=32, seed=53, n_inner_prefixes=3, random_durations=True,
                                       nthreads="random"), dict(n=2000, seed=54), 1.1, 0.3, 0, 0.0, 1),
        "svcgprio_c2mini_satinf": (dict(n=2500, w=24, seed=55), dict(n=1500, seed=56), float("inf"), 0.5, 0, 0.0, 1),
        # later graphs that depend on released earlier tasks: recomputed (recompute chains)
        "svcgrec_c2var_sat1.1": (dict(n=3000, w=32, seed=57, n_inner_prefixes=3, random_durations=True,
                                      nthreads="random"), dict(n=2000, seed=58), 1.1, 0.5, 0, 0.2, 0, True),
        "svcgrec_c2mini_satinf": (dict(n=2500, w=24, seed=59), dict(n=1500, seed=60), float("inf"), 0.6, 0, 0.3, 0,
                                  True),
    }
    for name, (a, b, sat, frac, *more) in cases.items():
        nadd = more[0] if more else 0
        dep_frac = more[1] if len(more) > 1 else 0.0
        user_prio = more[2] if len(more) > 2 else 0
        recompute = bool(more[3]) if len(more) > 3 else False
        if only and name not in only:
            continue
        kw = {k: v for k, v in a.items() if k not in ("n", "w", "seed", "restrict")}
        g = G.graphs.random_dag(a["n"], a["w"], seed=a["seed"], **kw)
        if a.get("restrict"):
            g = G.graphs.restrict(g, a["restrict"], seed=a["seed"], empty_frac=0.0)
        g2 = G.graphs.random_dag(b["n"], a["w"], seed=b["seed"], **kw)
        if b.get("restrict"):
            g2 = G.graphs.restrict(g2, b["restrict"], seed=b["seed"], empty_frac=0.1)
        g2["group_names"] = [nm.replace(G.graphs.TOKEN, TOKEN2) for nm in g2["group_names"]]
        assert g2["prefix_names"] == g["prefix_names"]
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        rec, rounds, nplaced, states, msgs, round_ptr, at, joins, ext = replay_second_graph(
            g, g2, cfg, 0, frac, nadd, dep_frac, restr=bool(b.get("restrict")), user_prio=user_prio, recompute=recompute)
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(msg_task=np.array(msgs["task"], np.int32), msg_worker=np.array(msgs["worker"], np.int32),
                 msg_runid=np.array(msgs["run_id"], np.int64), msg_nbytes=np.array(msgs["nbytes"], np.int64),
                 msg_start=np.array(msgs["start"]), msg_stop=np.array(msgs["stop"]),
                 msg_status=np.array(msgs["status"], np.int8), msg_round_ptr=np.array(round_ptr, np.int64),
                 g2_msg=np.array(at, np.int64))
        if nadd:
            z.update(add_msg=np.array(joins["msg"], np.int64), add_nthreads=np.array(joins["nthreads"], np.int32))
        for k in ("dep_ptr", "dep_idx", "prio", "prefix_id", "group_id", "wanted", "rootish_override"):
            z["g2_" + k] = np.asarray(g2[k])
        if user_prio:  # the merged ranks of every task (fixture order: the first graph's, then the later one's)
            z.update(g2_user_prio=np.array(user_prio, np.int64), g2_prio_all=ext["prio_all"])
        if dep_frac or b.get("restrict") or user_prio:  # dependencies on earlier tasks (-1 - t), placements, resync rows
            z.update(g2_dep_ptr=ext["ptr"], g2_dep_idx=ext["idx"], g2_nplaced=np.array(ext["nplaced"], np.int64),
                     **_pack_dumps(ext["dumps"]))
        if b.get("restrict"):
            z.update(g2_restr_ptr=np.asarray(g2["restr_ptr"]), g2_restr_idx=np.asarray(g2["restr_idx"]),
                     g2_restr_flags=np.asarray(g2["restr_flags"]))
        if recompute:  # the set-order rows of the recompute (distributed_amd/loss.py graph_orders)
            z.update(g2_lo_task=ext["lo_task"], g2_lo_kind=ext["lo_kind"], g2_lo_rowptr=ext["lo_rowptr"],
                     g2_lo_idx=ext["lo_idx"], g2_n_recomputed=np.array(ext["n_recomputed"], np.int64))
            print(f"{name}: {ext['n_recomputed']} earlier tasks recomputed, {len(ext['lo_task'])} order rows")
        np.savez_compressed(path, **z)
        routes = np.bincount(np.array(rec["route"]), minlength=4).tolist()
        print(f"{name}: {len(msgs['task'])} messages, second graph of {g2['n_tasks']} at message {at}, routes {routes}")


def _load_repo_module(name):
    import importlib.util

    spec = importlib.util.spec_from_file_location(f"dgp_{name}", os.path.join(G.REPO, "distributed_amd", f"{name}.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def later_graph(k, n, w, seed, n_prefixes):
    """Later graph k of a svcpfx_* stream: a C2-shaped random DAG whose task prefixes are its
    own (``g{k}root``, ``g{k}in{j}``: key_split keeps them) and whose groups carry a token of
    their own."""
    gk = G.graphs.random_dag(n, w, seed=seed, n_inner_prefixes=n_prefixes - 1, random_durations=True,
                             nthreads="random")
    names = [f"g{k}root"] + [f"g{k}in{j}" for j in range(n_prefixes - 1)]
    tok = f"{k:02d}" + TOKEN2[2:]
    gk["prefix_names"] = names
    gk["group_names"] = [f"{nm}-{tok}" for nm in names]
    return gk


def replay_later_graphs(g, later, cfg, at_fracs):
    """The replay protocol's completions as task-finished messages, with the independent
    graphs ``later`` submitted at the messages ``at_fracs`` of the first graph's size (as
    replay_second_graph submits one: new TaskStates of priority ``(0, 2 + k, i)``, then every
    new task recommended "waiting"). Each graph brings task prefixes of its own, so over the
    stream the session meets more of them than the engine's table holds (prefixes.PX). The
    engine's table follows the extension's rule (distributed_amd/prefixes.py, run here on the
    reference state at the point the extension's update_graph hook runs: the new TaskStates
    exist, released): a graph that fits appends its new names; one that does not compacts the
    table to the live prefixes, recorded as the remap (every earlier task's slot, each slot's
    default) plus the workers' and global resync rows in the new numbering."""
    P = _load_repo_module("prefixes")
    S = _load_repo_module("sync")
    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    W = len(g["nthreads"])
    N = g["n_tasks"]
    type(s).stimulus_task_finished = Scheduler_stimulus_task_finished()
    recs = {}
    for ts in sorted(tss, key=lambda t: t.priority, reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    nb, a0, b0 = list(g["nbytes"]), list(g["start"]), list(g["stop"])
    for gk in later:
        nb += list(gk["nbytes"])
        a0 += list(gk["start"])
        b0 += list(gk["stop"])
    cs = s.clients["client-0"]
    run_spec = (operator.add, (), {})
    # the extension's prefix bookkeeping (ext.py _note_prefixes / _add_graph / _compact_prefixes)
    slot_of = {nm: i for i, nm in enumerate(g["prefix_names"])}
    pnames = list(g["prefix_names"])
    pname_dur = {nm: float(d) for nm, d in zip(g["prefix_names"], g["prefix_default_dur"])}
    task_pname = np.asarray(g["prefix_id"], np.int32).copy()
    group_names = list(g["group_names"])
    at_msgs = [int(f * N) for f in at_fracs]
    subs = []  # per later graph: message index, its prefix ids (engine slots), the table's defaults, the remap

    def submit(k):
        nonlocal slot_of, task_pname
        gk = later[k]
        base = len(tss)
        keys_k = G.make_keys(gk)
        new = []
        for t, key in enumerate(keys_k):
            ts = s.new_task(key, run_spec, "released")
            tidx[key] = base + t
            ts.priority = (0, 2 + k, int(gk["prio"][t]))
            new.append(ts)
        ptr, idx = gk["dep_ptr"], gk["dep_idx"]
        for t, ts in enumerate(new):
            for d in idx[ptr[t]:ptr[t + 1]]:
                ts.add_dependency(new[int(d)])
            if gk["wanted"][t]:
                ts.who_wants = {cs}
                cs.wants_what.add(ts)
        # the extension's hook: the graph's names in the order its ingestion meets them (the
        # new tasks in priority order), then the table
        order = np.argsort(np.asarray(gk["prio"]), kind="stable")
        first = []
        for t in order.tolist():
            nm = gk["prefix_names"][int(gk["prefix_id"][t])]
            if nm not in first:
                first.append(nm)
        sub = {"msg": None, "remap": None}
        if len(slot_of) + sum(nm not in slot_of for nm in first) > P.PX:
            live = P.live_prefixes(s)
            table = P.compacted(slot_of, live, first)
            assert table is not None, f"more than PX live prefixes: {len(live)} live + {first}"
            slots, stale = P.task_slots(task_pname, pnames, table)
            names = sorted(table, key=table.get)
            defaults = [pname_dur.get(nm, -1.0) for nm in names]
            keys_old = [ts.key for ts in tss]
            workers = [a for a, _ in sorted(widx.items(), key=lambda kv: kv[1])]
            sub["remap"] = dict(slots=slots, defaults=np.array(defaults, np.float64),
                                workers=S.worker_rows(s, workers, table, {k_: tidx[k_] for k_ in keys_old}),
                                globals=S.global_rows(s, names, defaults, group_names,
                                                      {k_: tidx[k_] for k_ in keys_old}, widx))
            slot_of = table
        for nm in first:
            if nm not in slot_of:
                slot_of[nm] = len(slot_of)
        for nm, d in zip(gk["prefix_names"], gk["prefix_default_dur"]):
            if nm not in pname_dur:
                pname_dur[nm] = float(d)
                pnames.append(nm)
        names_now = sorted(slot_of, key=slot_of.get)
        sub["prefix_id"] = np.array([slot_of[gk["prefix_names"][int(p)]] for p in gk["prefix_id"]], np.int32)
        sub["defaults"] = np.array([pname_dur.get(nm, -1.0) for nm in names_now], np.float64)
        sub["group_base"] = len(group_names)
        group_names.extend(gk["group_names"])
        pid = {nm: i for i, nm in enumerate(pnames)}
        task_pname = np.concatenate([task_pname, np.array([pid[gk["prefix_names"][int(p)]] for p in gk["prefix_id"]],
                                                          np.int32)])
        recs2 = {ts.key: "waiting" for ts in sorted(new, key=lambda t: t.priority, reverse=True)}
        s._transitions(recs2, {}, {}, f"update-graph-{k + 2}")
        tss.extend(new)
        subs.append(sub)

    msgs = {k: [] for k in ("task", "worker", "run_id", "nbytes", "start", "stop", "status")}
    stim = [len(rec["task"])]
    round_ptr = [0]
    rounds, nplaced = [], []
    done = 0
    nsub = 0
    while True:
        cur = len(rec["task"])
        batch = list(range(done, cur))
        rounds.append(G.snapshot(s, W, widx) + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for pos in batch:
            while nsub < len(later) and len(msgs["task"]) >= at_msgs[nsub]:
                n0 = len(rec["task"])
                submit(nsub)
                subs[-1]["msg"] = len(msgs["task"])
                subs[-1]["nplaced"] = len(rec["task"]) - n0
                stim.append(len(rec["task"]) - n0)
                nsub += 1
            t = rec["task"][pos]
            ts = tss[t]
            assert ts.state == "processing", (ts.key, ts.state)
            w = widx[ts.processing_on.address]
            sid = f"task-finished-{len(msgs['task'])}"
            r, cm, wm = s.stimulus_task_finished(
                ts.key, ts.processing_on.address, sid, int(ts.run_id), nbytes=int(nb[t]), type=None,
                typename="int", metadata=None,
                startstops=[{"action": "compute", "start": float(a0[t]), "stop": float(b0[t])}])
            n0 = len(rec["task"])
            s._transitions(r, cm, wm, sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
            stim.append(len(rec["task"]) - n0)
            for k, v in zip(("task", "worker", "run_id", "nbytes", "start", "stop", "status"),
                            (t, w, pos, int(nb[t]), float(a0[t]), float(b0[t]), ACCEPTED)):
                msgs[k].append(v)
        round_ptr.append(len(msgs["task"]))
    assert nsub == len(later), (nsub, len(later))
    rec["stim"] = stim
    states = np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8)
    return rec, rounds, nplaced, states, msgs, round_ptr, subs, len(pnames)


def Scheduler_stimulus_task_finished():
    from distributed.scheduler import Scheduler

    return Scheduler.stimulus_task_finished


def main_prefixes(only):
    """svcpfx_*: later graphs with task prefixes of their own, more over the stream than the
    engine's table (prefixes.PX) -- the table compacts to the live prefixes."""
    cases = {
        # 3 + 6 x 12 = 75 task prefixes over the stream, at most ~27 live at once
        "svcpfx_c2var_sat1.1": (dict(n=3000, w=32, seed=61, n_inner_prefixes=2), 6, 500, 12, 1.1),
        "svcpfx_c2var_satinf": (dict(n=2500, w=24, seed=62, n_inner_prefixes=2), 6, 400, 12, float("inf")),
    }
    for name, (a, K, nk, pk, sat) in cases.items():
        if only and name not in only:
            continue
        g = G.graphs.random_dag(a["n"], a["w"], seed=a["seed"], n_inner_prefixes=a["n_inner_prefixes"],
                                random_durations=True, nthreads="random")
        later = [later_graph(k, nk, a["w"], a["seed"] * 10 + k, pk) for k in range(K)]
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        at = [0.1 + 0.3 * k for k in range(K)]  # message indices (x the first graph's size)
        rec, rounds, nplaced, states, msgs, round_ptr, subs, n_names = replay_later_graphs(g, later, cfg, at)
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(msg_task=np.array(msgs["task"], np.int32), msg_worker=np.array(msgs["worker"], np.int32),
                 msg_runid=np.array(msgs["run_id"], np.int64), msg_nbytes=np.array(msgs["nbytes"], np.int64),
                 msg_start=np.array(msgs["start"]), msg_stop=np.array(msgs["stop"]),
                 msg_status=np.array(msgs["status"], np.int8), msg_round_ptr=np.array(round_ptr, np.int64),
                 gk_n=np.array(K, np.int64), gk_prefix_names_total=np.array(n_names, np.int64))
        dumps = []
        for k, (gk, sub) in enumerate(zip(later, subs)):
            p = f"g{k}_"
            for f in ("dep_ptr", "dep_idx", "prio", "group_id", "wanted", "rootish_override", "nbytes", "start",
                      "stop"):
                z[p + f] = np.asarray(gk[f])
            z[p + "prefix_id"] = sub["prefix_id"]  # the engine's slots
            z[p + "prefix_local"] = np.asarray(gk["prefix_id"], np.int32)  # into its own names
            z[p + "prefix_names"] = np.array(gk["prefix_names"])
            z[p + "group_names"] = np.array(gk["group_names"])
            z[p + "group_local"] = np.asarray(gk["group_id"], np.int32)
            z[p + "group_id"] = np.asarray(gk["group_id"], np.int32) + sub["group_base"]
            z[p + "defaults"] = sub["defaults"]
            z[p + "msg"] = np.array(sub["msg"], np.int64)
            z[p + "nplaced"] = np.array(sub["nplaced"], np.int64)
            z[p + "n_groups"] = np.array(sub["group_base"] + len(gk["group_names"]), np.int64)
            if sub["remap"] is not None:
                z[p + "remap_slots"] = sub["remap"]["slots"]
                z[p + "remap_defaults"] = sub["remap"]["defaults"]
                z[p + "remap_dump"] = np.array(len(dumps), np.int64)
                dumps.append(dict(tasks=dict(task=np.zeros(0, np.int32)), workers=sub["remap"]["workers"],
                                  globals=sub["remap"]["globals"]))
        if dumps:
            z.update({k_: v for k_, v in _pack_dumps(dumps).items() if not k_.startswith("sync_tasks")})
        np.savez_compressed(path, **z)
        nrm = sum(sub["remap"] is not None for sub in subs)
        print(f"{name}: {len(msgs['task'])} messages, {K} later graphs, {n_names} task prefixes, {nrm} remaps, "
              f"{len(rec['task'])} placements")


# event kinds of the svcev_* streams (tests/test_gpu_events.py, tests/ext_driver.py)
EV_FINISHED, EV_ADD_KEYS, EV_RELEASE_DATA, EV_PAUSE, EV_RESUME, EV_LONG_RUNNING, EV_HEARTBEAT, EV_ERRED = range(8)
# stimuli the engine does not model: the scheduler decides them, then the engine resyncs
# (dgp_sync_*; the fixture stores the scheduler's state after each, distributed_amd/sync.py)
EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS = 8, 9, 10
RESYNC_KINDS = (EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS)
# the P2P shuffle's scheduler-side lifecycle (svcp2p_*): placement inputs its plugin changes
# outside any transition (shuffle/_scheduler_plugin.py); the tasks of an init are in hb_task
EV_SHUFFLE_INIT, EV_RESTRICT = 11, 12
# a drained worker retires (svcrt_*): retire_workers' shape -- paused, its processing done, its
# sole replicas copied elsewhere by add-keys -- then Scheduler.remove_worker, which runs no
# transition; EV_RETIRE_REPLICA records each replica remove_worker drops there (has_what
# order), EV_RETIRE the removal itself. The engine follows it without a resync.
EV_RETIRE, EV_RETIRE_REPLICA = 13, 14
# a worker with processing tasks or sole replicas is lost (svcwl_*): Scheduler.remove_worker
# releases and re-places its processing tasks and recomputes its lost results; the engine
# decides the whole stimulus (dgp_lose_worker). hb_task holds the worker's processing tasks
# in ws.processing iteration order (ev_x of them), then its replicas in ws.has_what order.
EV_LOSE_WORKER = 15
# a task-erred that does not err (svcretry_*): a retry (ts.retries > 0, ev_x 0) or a stale run's
# report from the worker it runs on (ev_x 1) of a task something needs -- stimulus_task_erred
# :5111-5118 and its transitions (processing -> released -> waiting -> decide_worker), then
# handle_task_erred's queue refill (:5805) as the EV_REFILL event that follows it
EV_ERRED_RETRY, EV_REFILL = 16, 17


def _loss_is_supported(s, ws):
    """The worker losses the engine decides itself (dgp_lose_worker; the extension checks the
    same before it asks): no processing task that errs
    (KilledWorker) or that nobody needs, and every lost result that is needed has its
    dependencies in memory elsewhere and no queued / no-worker dependent."""
    for ts in ws.processing:
        if ts.suspicious + 1 > s.allowed_failures or not (ts.waiters or ts.who_wants) or ts.has_lost_dependencies:
            return False
    for ts in ws.has_what:
        if ts.who_has != {ws}:
            continue
        if not ts.run_spec or ts.has_lost_dependencies:
            return False
        if ts.who_wants or ts.waiters:
            for d in ts.dependencies:
                if d.state != "memory" or d.who_has == {ws}:
                    return False
        for d in ts.waiters or ():
            if d.state in ("queued", "no-worker"):
                return False
            if d.state == "processing" and not (d.waiters or d.who_wants):
                return False
    return True


def _dump(s, g, tidx, widx, keys):
    """The scheduler's state as the engine's resync rows (every task of the graph)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("dgp_sync", os.path.join(G.REPO, "distributed_amd", "sync.py"))
    S = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(S)
    workers = [a for a, _ in sorted(widx.items(), key=lambda kv: kv[1])]
    return dict(tasks=S.task_rows(s, keys, tidx, widx),
                workers=S.worker_rows(s, workers, {nm: i for i, nm in enumerate(g["prefix_names"])}, tidx),
                globals=S.global_rows(s, list(g["prefix_names"]), list(g["prefix_default_dur"]),
                                      list(g["group_names"]), tidx, widx))


def _pack_dumps(dumps):
    """The dumps of one fixture as arrays: sync_<part>_<field> concatenated over the dumps
    with sync_<part>_<field>_ptr (each dump's slice)."""
    out = {}
    for part in ("tasks", "workers", "globals"):
        for field in dumps[0][part]:
            vals = [np.atleast_1d(np.asarray(d[part][field])) for d in dumps]
            ptr = np.zeros(len(vals) + 1, np.int64)
            ptr[1:] = np.cumsum([len(v) for v in vals])
            out[f"sync_{part}_{field}"] = np.concatenate(vals)
            out[f"sync_{part}_{field}_ptr"] = ptr
    return out


def _erred_is_simple(s, ts):
    """The task-erred cascade of ``ts`` (stimulus_task_erred :5094 -> processing -> erred
    :2630-2720, its waiting dependents released then erred :2579-2605 / :2508-2537) releases
    only dependencies that are in memory: a cascade that would also cancel processing,
    waiting or queued tasks is not generated (the engine refuses it)."""
    closure, stack = {ts}, [ts]
    while stack:
        x = stack.pop()
        for y in x.dependents:
            if y not in closure and not y.who_has:
                closure.add(y)
                stack.append(y)
    for x in closure:
        for d in x.dependencies:
            if d in closure:
                if d is not ts and not d.who_wants:  # x's release may override d's "erred" (dgp_events.h)
                    return False
                continue
            if not (d.waiters or set()) - closure and not d.who_wants and d.state != "memory":
                return False
    return all(x is ts or x.state == "waiting" for x in closure)


def replay_events(g, cfg, seed, p_event=0.08, kinds=(1, 2, 3, 4, 5, 6, 7), bw_scale=0.3, dumps=None, chains=False,
                  allowed_failures=3, release_memory=False, release_cancel=False):
    """The replay protocol's completions as task-finished messages, interleaved with the
    other worker stimuli that change placement inputs, each through the reference's own
    handler (``Scheduler.*`` borrowed onto the replay state):

    * add-keys (``Scheduler.add_keys`` :7359-7391 -> ``add_replica`` :3148): a replica of an
      in-memory task on a worker that does not hold it;
    * release-worker-data (``Scheduler.release_worker_data`` :5807-5815): one of several
      replicas goes (never the last: that recomputes);
    * worker-status-change (``Scheduler.handle_worker_status_change`` :5850-5883): a running
      worker pauses / a paused one runs again (check_idle_saturated, refill);
    * long-running (``Scheduler.handle_long_running`` :5817-5848): a processing task
      secedes, with a compute duration or None;
    * heartbeat (``Scheduler.heartbeat_worker``'s placement part, restated line by line:
      the bandwidth EWMA :4223-4226 and TaskPrefix.add_exec_time for the executing tasks
      :4247-4252);
    * task-erred (``Scheduler.handle_task_erred`` :5799-5805 -> ``stimulus_task_erred``
      :5094-5127) of a current run (no retries), when its cascade releases only in-memory
      dependencies (``_erred_is_simple``); the erred task sends no task-finished.

    Stored per event (``ev_*``, in order): kind, task, worker, a float (long-running
    compute duration, NaN for None; heartbeat: the scheduler bandwidth after it), the
    heartbeat's executing tasks and durations (CSR ``hb_ptr`` / ``hb_task`` / ``hb_dur``), and
    the placements each event made (``stim_nplaced``: update_graph first).

    ``chains``: worker losses may recompute released dependencies and err tasks out of retries
    (KilledWorker: ``allowed_failures``), as distributed_amd/loss.py accepts them; each loss
    event's order rows (the set orders the cascade follows, as loss_orders gives them in this
    process) go to ``hb["lo"]``: CSR over events (``evptr``) into rows (``task``, ``kind``,
    ``rowptr`` into ``idx``), and its killed processing tasks (``kptr`` into ``ktask``)."""
    from distributed.scheduler import Scheduler

    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    W = len(g["nthreads"])
    N = g["n_tasks"]
    addr = {i: a for a, i in widx.items()}
    rng = np.random.default_rng(seed)
    S = type(s)
    S.stimulus_task_finished = Scheduler.stimulus_task_finished
    S.add_keys = Scheduler.add_keys
    S.release_worker_data = Scheduler.release_worker_data
    S.handle_worker_status_change = Scheduler.handle_worker_status_change
    S.handle_long_running = Scheduler.handle_long_running
    S.handle_task_erred = Scheduler.handle_task_erred
    S.stimulus_task_erred = Scheduler.stimulus_task_erred
    S.send_all = lambda self, client_msgs, worker_msgs: None
    S.worker_send = lambda self, worker, msg: None
    s.extensions = {}
    if EV_REMOVE_WORKER in kinds or EV_RETIRE in kinds or EV_LOSE_WORKER in kinds:  # what Scheduler.remove_worker touches besides placement state
        import asyncio
        from collections import defaultdict
        from types import SimpleNamespace as NS

        from distributed.core import Status
        from distributed.comm.addressing import get_address_host

        S.remove_worker = Scheduler.remove_worker
        S.transition = Scheduler.transition  # a KilledWorker's processing -> erred (:5249-5256)
        S.remove_resources = lambda self, address: None
        S.coerce_address = lambda self, a, resolve=True: a
        s.status = Status.running
        s.stream_comms = defaultdict(lambda: NS(send=lambda msg: None))
        s.rpc = NS(remove=lambda a: None)
        s.host_info = {}
        for a, ws in s.workers.items():
            h = s.host_info.setdefault(get_address_host(a), {"addresses": set(), "nthreads": 0})
            h["addresses"].add(a)
            h["nthreads"] += ws.nthreads
        s.total_nthreads_history = []
        s.allowed_failures = allowed_failures
        s.bandwidth_workers = {}
        s.events = {}
        s._ongoing_background_tasks = NS(closed=False, call_later=lambda *a, **k: None)
        loop = asyncio.new_event_loop()
    if EV_RESCHEDULE in kinds:
        S._reschedule = Scheduler._reschedule
    if EV_RELEASE_KEYS in kinds:
        S.client_releases_keys = Scheduler.client_releases_keys
    removed = set()
    recs = {}
    for ts in sorted(tss, key=lambda t: t.priority, reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    ev = {k: [] for k in ("kind", "task", "worker", "x", "nbytes", "start", "stop", "runid")}
    hb = {"ptr": [0], "task": [], "dur": []}
    lo = {"evptr": [0], "task": [], "kind": [], "rowptr": [0], "idx": [], "kptr": [0], "ktask": [],
          "rptr": [0], "rtask": [], "rforget": []}
    hb["lo"] = lo
    LS = _load_repo_module("loss") if chains else None
    stim = [len(rec["task"])]
    round_ptr = [0]
    rounds, nplaced = [], []
    done = 0
    erred = set()
    paused = set()

    def push(kind, t=-1, w=-1, x=math.nan, nbytes=-1, start=math.nan, stop=math.nan, runid=-1):
        for k, v in zip(ev, (kind, t, w, x, nbytes, start, stop, runid)):
            ev[k].append(v)
        hb["ptr"].append(len(hb["task"]))
        lo["evptr"].append(len(lo["task"]))
        lo["kptr"].append(len(lo["ktask"]))
        lo["rptr"].append(len(lo["rtask"]))

    def event():
        kind = int(rng.choice(kinds))
        sid = f"event-{len(ev['kind'])}"
        n0 = len(rec["task"])
        if kind == EV_ADD_KEYS:
            mem = [ts for ts in tss if ts.state == "memory"]
            if not mem:
                return
            ts = mem[int(rng.integers(0, len(mem)))]
            others = [i for i in range(W) if i not in removed and s.workers[addr[i]] not in ts.who_has]
            if not others:
                return
            w = others[int(rng.integers(0, len(others)))]
            s.add_keys(worker=addr[w], keys=[ts.key], stimulus_id=sid)
            push(EV_ADD_KEYS, tidx[ts.key], w)
        elif kind == EV_RELEASE_DATA:
            rep = [ts for ts in tss if ts.state == "memory" and len(ts.who_has) >= 2]
            if not rep:
                return
            ts = rep[int(rng.integers(0, len(rep)))]
            hs = sorted(widx[ws.address] for ws in ts.who_has)
            w = hs[int(rng.integers(0, len(hs)))]
            s.release_worker_data(ts.key, addr[w], sid)
            push(EV_RELEASE_DATA, tidx[ts.key], w)
        elif kind == EV_PAUSE:
            run = [i for i in range(W) if i not in paused and i not in removed]
            if len(run) <= max(1, W // 2):
                return
            w = run[int(rng.integers(0, len(run)))]
            s.handle_worker_status_change("paused", addr[w], sid)
            paused.add(w)
            push(EV_PAUSE, -1, w)
        elif kind == EV_RESUME:
            if not paused:
                return
            ps = sorted(paused)
            w = ps[int(rng.integers(0, len(ps)))]
            s.handle_worker_status_change("running", addr[w], sid)
            paused.discard(w)
            push(EV_RESUME, -1, w)
        elif kind == EV_LONG_RUNNING:
            proc = [ts for ts in tss if ts.state == "processing" and ts not in ts.processing_on.long_running]
            if not proc:
                return
            ts = proc[int(rng.integers(0, len(proc)))]
            cd = None if rng.random() < 0.3 else float(rng.uniform(0.001, 0.05))
            s.handle_long_running(ts.key, ts.processing_on.address, cd, sid)
            push(EV_LONG_RUNNING, tidx[ts.key], widx[ts.processing_on.address], math.nan if cd is None else cd)
        elif kind == EV_HEARTBEAT:
            w = int(rng.integers(0, W))
            if w in removed:
                return
            ws = s.workers[addr[w]]
            total = float(rng.uniform(1 - bw_scale, 1 + bw_scale) * 1e8)
            # Scheduler.heartbeat_worker :4223-4226 (bandwidth EWMA)
            frac = 1 / len(s.workers)
            s.bandwidth = s.bandwidth * (1 - frac) + total * frac
            # :4247-4252 (the executing tasks' prefixes see their exec time)
            execs = [ts for ts in ws.processing]
            execs.sort(key=lambda t: tidx[t.key])
            k = int(rng.integers(0, min(3, len(execs)) + 1))
            for ts in execs[:k]:
                d = float(rng.choice([rng.uniform(0.0, 0.02), rng.uniform(0.02, 2.0)]))
                ts.prefix.add_exec_time(d)
                hb["task"].append(tidx[ts.key])
                hb["dur"].append(d)
            push(EV_HEARTBEAT, -1, w, s.bandwidth)
        elif kind == EV_REMOVE_WORKER:
            live = [i for i in range(W) if i not in removed and i not in paused]
            if len(live) <= max(2, W // 2):
                return
            w = live[int(rng.integers(0, len(live)))]
            loop.run_until_complete(s.remove_worker(addr[w], stimulus_id=sid))
            removed.add(w)
            push(EV_REMOVE_WORKER, -1, w)
        elif kind == EV_LOSE_WORKER:
            live = [i for i in range(W) if i not in removed]
            if len(live) <= max(2, W // 2):
                return
            cand, chained, casc = [], [], {}
            for i in live:
                ws = s.workers[addr[i]]
                busy = bool(ws.processing) or any(ts.who_has == {ws} for ts in ws.has_what)
                if not busy:
                    continue
                if chains:
                    c = LS.supported(s, ws, list(ws.processing), list(ws.has_what), False)
                    if c is not None:
                        cand.append(i)
                        casc[i] = c
                        # recomputes a released dependency, or errs a task out of retries
                        if any(t.state == "released" for t in c[0]) or c[1]:
                            chained.append(i)
                elif _loss_is_supported(s, ws):
                    cand.append(i)
            if not cand:
                return
            pick = chained if chained and rng.random() < 0.75 else cand
            w = pick[int(rng.integers(0, len(pick)))]
            ws = s.workers[addr[w]]
            if chains:
                kf = LS.killed_flags(s, list(ws.processing), False)
                for t, k, seq in LS.loss_orders(casc[w][0], lambda ts: tidx[ts.key], casc[w][1], sum(kf)):
                    lo["task"].append(t)
                    lo["kind"].append(k)
                    lo["idx"].extend(seq)
                    lo["rowptr"].append(len(lo["idx"]))
                lo["ktask"].extend(tidx[ts.key] for ts, k in zip(ws.processing, kf) if k)
            proc = [tidx[ts.key] for ts in ws.processing]  # the order remove_worker iterates (:5236)
            held = [tidx[ts.key] for ts in ws.has_what]  # ... and :5270
            if os.environ.get("DGP_DEBUG_STATES"):
                watch = [int(x) for x in os.environ["DGP_DEBUG_STATES"].split(",") if x]
                before = {t: (tss[t].state, sorted(widx[h.address] for h in tss[t].who_has or ()),
                              len(tss[t].waiters or ())) for t in watch}
            loop.run_until_complete(s.remove_worker(addr[w], stimulus_id=sid))
            if os.environ.get("DGP_DEBUG_STATES"):
                print("LOSS", len(hb.get("dbg", [])), "worker", w, "proc", proc, "held", held, flush=True)
                for t in watch:
                    print("   ", t, before[t], "->", (tss[t].state, sorted(widx[h.address] for h in tss[t].who_has or ()),
                                                     len(tss[t].waiters or ())), flush=True)
            removed.add(w)
            paused.discard(w)
            hb["task"].extend(proc + held)
            hb["dur"].extend([0.0] * (len(proc) + len(held)))
            push(EV_LOSE_WORKER, -1, w, float(len(proc)))
            if os.environ.get("DGP_DEBUG_STATES"):  # diagnostics: the states after each loss
                hb.setdefault("dbg", []).append(np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8))
        elif kind == EV_RETIRE:
            cand = [i for i in sorted(paused) if i not in removed and not s.workers[addr[i]].processing]
            live = [i for i in range(W) if i not in removed and i not in paused]
            if not cand or len(live) <= max(2, W // 2):
                return
            w = cand[int(rng.integers(0, len(cand)))]
            ws = s.workers[addr[w]]
            for ts in list(ws.has_what):  # retire_workers' replicate step: no last replica leaves
                if len(ts.who_has) == 1:
                    w2 = live[int(rng.integers(0, len(live)))]
                    s.add_keys(worker=addr[w2], keys=[ts.key], stimulus_id=sid)
                    push(EV_ADD_KEYS, tidx[ts.key], w2)
                    stim.append(0)
            held = [tidx[ts.key] for ts in ws.has_what]
            loop.run_until_complete(s.remove_worker(addr[w], stimulus_id=sid))
            assert len(rec["task"]) == n0  # no transition ran, nothing was placed
            removed.add(w)
            paused.discard(w)
            for t in held:
                push(EV_RETIRE_REPLICA, t, w)
                stim.append(0)
            push(EV_RETIRE, -1, w)
        elif kind == EV_RESCHEDULE:
            proc = [ts for ts in tss if ts.state == "processing"]
            if not proc:
                return
            ts = proc[int(rng.integers(0, len(proc)))]
            w = widx[ts.processing_on.address]
            s._reschedule(ts.key, addr[w], stimulus_id=sid)
            push(EV_RESCHEDULE, tidx[ts.key], w)
        elif kind == EV_RELEASE_KEYS:
            states = (("memory",) if release_memory else
                      ("waiting", "processing", "queued", "no-worker", "memory") if release_cancel else
                      ("waiting", "processing", "queued"))
            wanted = [ts for ts in tss if ts.who_wants and ts.state in states]
            if not wanted:
                return
            ts = wanted[int(rng.integers(0, len(wanted)))]
            if release_memory or release_cancel:  # what the engine takes (loss.release_plan, as the extension)
                LR = _load_repo_module("loss")
                plan = LR.release_plan(s, "client-0", [ts.key])
                for _ in range(32 if release_cancel else 0):  # a release the engine restates
                    if plan is not None:
                        break
                    ts = wanted[int(rng.integers(0, len(wanted)))]
                    plan = LR.release_plan(s, "client-0", [ts.key])
                if plan is None and release_cancel:
                    return
                assert plan is not None, ts.key
                for x, f in plan:
                    lo["rtask"].append(tidx[x.key])
                    lo["rforget"].append(1 if f else 0)
            before = [x.state for x in tss] if release_cancel else None
            s.client_releases_keys(keys=[ts.key], client="client-0", stimulus_id=sid)
            if release_cancel:  # the plan names exactly the tasks the transitions changed (the refill aside)
                ops = {tidx[x.key] for x, _ in plan}
                chg = {i for i, x in enumerate(tss) if x.state != before[i] and not
                       (before[i] == "queued" and x.state == "processing")}
                assert chg == ops, (sorted(chg - ops)[:8], sorted(ops - chg)[:8],
                                    [(i, before[i], tss[i].state) for i in sorted(chg ^ ops)[:8]])
            push(EV_RELEASE_KEYS, tidx[ts.key], -1)
        elif kind == EV_ERRED_RETRY:
            proc = [ts for ts in tss if ts.state == "processing" and (ts.waiters or ts.who_wants)
                    and not ts.has_lost_dependencies]
            if not proc:
                return
            ts = proc[int(rng.integers(0, len(proc)))]
            w = widx[ts.processing_on.address]
            stale = bool(rng.random() < 0.3)
            if not stale:
                ts.retries = 1
            run = ts.run_id - 1 if stale else ts.run_id
            # Scheduler.handle_task_erred (:5799-5805), its two parts as two events
            r = s.stimulus_task_erred(key=ts.key, stimulus_id=sid, worker=addr[w], run_id=run, exception=None,
                                      traceback=None)
            s._transitions(r[0], r[1], r[2], sid)
            assert ts.state != "erred", ts.state
            push(EV_ERRED_RETRY, tidx[ts.key], w, 1.0 if stale else 0.0, runid=run)
            stim.append(len(rec["task"]) - n0)
            n0 = len(rec["task"])
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
            push(EV_REFILL)
        elif kind == EV_ERRED:
            proc = [ts for ts in tss if ts.state == "processing" and _erred_is_simple(s, ts)]
            if not proc:
                return
            ts = proc[int(rng.integers(0, len(proc)))]
            w = widx[ts.processing_on.address]
            s.handle_task_erred(key=ts.key, stimulus_id=sid, worker=addr[w], run_id=ts.run_id, exception=None,
                                traceback=None)
            assert ts.state == "erred", ts.state
            erred.add(tidx[ts.key])
            push(EV_ERRED, tidx[ts.key], w)
        if kind in RESYNC_KINDS and ev["kind"] and ev["kind"][-1] == kind:
            dumps.append(_dump(s, g, tidx, widx, [ts.key for ts in tss]))
        stim.append(len(rec["task"]) - n0)

    run_of = []  # the reference run_id of each placement-log entry
    orig_add = S._add_to_processing

    def add_to_processing(self, ts, ws, stimulus_id):
        r = orig_add(self, ts, ws, stimulus_id)
        run_of.append(int(ts.run_id))
        return r

    S._add_to_processing = add_to_processing
    run_of.extend([int(tss[t].run_id) for t in rec["task"]])  # update_graph's, already made
    # the compute-task messages the reference builds from here on (_task_to_msg :3421-3450),
    # one per placement-log entry: who_has (holder indices, ascending) and nbytes per
    # dependency, in the graph's dep_idx order
    n_ug = len(rec["task"])
    tm = {"task": [], "dep_ptr": [0], "dep_task": [], "dep_nbytes": [], "hold_ptr": [0], "hold_idx": []}
    orig_msg = S._task_to_msg
    dp, di = g["dep_ptr"], g["dep_idx"]

    def task_to_msg(self, ts, duration=-1):
        m = orig_msg(self, ts, duration)
        t = tidx[ts.key]
        deps = di[dp[t]:dp[t + 1]].tolist()
        assert sorted(tidx[k] for k in m["who_has"]) == sorted(deps) == sorted(tidx[k] for k in m["nbytes"])
        tm["task"].append(t)
        for d in deps:
            k = tss[d].key
            tm["dep_task"].append(d)
            tm["dep_nbytes"].append(int(m["nbytes"][k]))
            tm["hold_idx"].extend(sorted(widx[a] for a in m["who_has"][k]))
            tm["hold_ptr"].append(len(tm["hold_idx"]))
        tm["dep_ptr"].append(len(tm["dep_task"]))
        return m

    S._task_to_msg = task_to_msg
    while True:
        cur = len(rec["task"])
        batch = list(range(done, cur))
        rounds.append(G.snapshot(s, W, widx) + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for pos in batch:
            while rng.random() < p_event:
                event()
            t = rec["task"][pos]
            ts = tss[t]
            if ts.state != "processing":  # erred, released by a client, or re-placed (a later entry)
                continue
            if int(ts.run_id) != run_of[pos]:  # a later placement of the same task completes it
                continue
            w = widx[ts.processing_on.address]
            sid = f"task-finished-{len(ev['kind'])}"
            r, cm, wm = s.stimulus_task_finished(
                ts.key, ts.processing_on.address, sid, int(ts.run_id), nbytes=int(g["nbytes"][t]), type=None,
                typename="int", metadata=None,
                startstops=[{"action": "compute", "start": float(g["start"][t]), "stop": float(g["stop"][t])}])
            assert ts.state != "processing"
            n0 = len(rec["task"])
            s._transitions(r, cm, wm, sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
            stim.append(len(rec["task"]) - n0)
            push(EV_FINISHED, t, w, math.nan, int(g["nbytes"][t]), float(g["start"][t]), float(g["stop"][t]), pos)
        round_ptr.append(len(ev["kind"]))
    rec["stim"] = stim
    S._task_to_msg = orig_msg
    assert len(tm["task"]) == len(rec["task"]) - n_ug and tm["task"] == rec["task"][n_ug:]
    ev["tm"] = dict(tm, first=n_ug)
    states = np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8)
    if os.environ.get("DGP_DEBUG_STORY"):  # diagnostics: the transitions of the named tasks
        for q in [int(x) for x in os.environ["DGP_DEBUG_STORY"].split(",") if x]:
            for e in s.story(tss[q].key):
                print("STORY", q, tss[q].key, e[0] == tss[q].key, e[1], e[2], e[4], flush=True)
    return rec, rounds, nplaced, states, ev, hb, round_ptr


def _tm_arrays(tm):
    """The recorded compute-task messages as fixture arrays (tm_*)."""
    return dict(tm_first=np.int64(tm["first"]), tm_task=np.array(tm["task"], np.int32),
                tm_dep_ptr=np.array(tm["dep_ptr"], np.int64), tm_dep_task=np.array(tm["dep_task"], np.int32),
                tm_dep_nbytes=np.array(tm["dep_nbytes"], np.int64), tm_hold_ptr=np.array(tm["hold_ptr"], np.int64),
                tm_hold_idx=np.array(tm["hold_idx"], np.int32))


def replay_p2p(g, cfg, dumps):
    """The P2P shuffle's scheduler-side lifecycle on the shuffle graph as the client submits
    it (graphs.shuffle_graph(live=True): the unpacks' _rootish None, no restrictions), each
    step through the reference's own code (``ShuffleSchedulerPlugin`` bound to this state):

    1. the transfers run; when the first one starts (shuffle_get_or_create -> ``_create``)
       ``_ensure_output_tasks_are_non_rootish`` sets ``_rootish = False`` on every unpack
       (shuffle/_scheduler_plugin.py:140-151, :254-278) -- EV_SHUFFLE_INIT;
    2. the barrier completes; the unpacks go by decide_worker_non_rootish to its holder;
    3. each unpack runs once: ``restrict_task`` -> ``_set_restriction`` ->
       ``Scheduler.set_restrictions({key: {worker}})`` (:101-115, :281-293;
       scheduler.py:7702-7707) with the range-sharded worker (shuffle/_shuffle.py:612-617)
       -- EV_RESTRICT -- then raises Reschedule: ``Scheduler._reschedule`` (the "reschedule"
       stream handler) re-places it under the restriction -- EV_RESCHEDULE, a resync dump;
    4. the re-placed unpacks complete.

    Everything else is the replay protocol (completions in placement-log order)."""
    from types import SimpleNamespace as NS

    from distributed.scheduler import Scheduler
    from distributed.shuffle._core import barrier_key
    from distributed.shuffle._scheduler_plugin import ShuffleSchedulerPlugin
    from distributed.shuffle._shuffle import _get_worker_for_range_sharding

    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    W = len(g["nthreads"])
    N = g["n_tasks"]
    P = (N - 1) // 3
    addr = {i: a for a, i in widx.items()}
    S = type(s)
    S.stimulus_task_finished = Scheduler.stimulus_task_finished
    S.set_restrictions = Scheduler.set_restrictions
    S._reschedule = Scheduler._reschedule
    S.send_all = lambda self, client_msgs, worker_msgs: None
    S.worker_send = lambda self, worker, msg: None
    s.extensions = {}
    transfers = set(range(P, 2 * P))
    bar = tss[2 * P]
    # the plugin, bound to this state: its barrier lookup by name (barrier_key) finds the
    # fixture's barrier task
    sid = "fixture"
    plugin = ShuffleSchedulerPlugin.__new__(ShuffleSchedulerPlugin)
    plugin.scheduler = NS(tasks={barrier_key(sid): bar}, set_restrictions=s.set_restrictions)
    spec = NS(id=sid)
    recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    s._transitions(recs, {}, {}, "update-graph")
    ev = {k: [] for k in ("kind", "task", "worker", "x", "nbytes", "start", "stop", "runid")}
    hb = {"ptr": [0], "task": [], "dur": []}
    lo = {"evptr": [0], "task": [], "kind": [], "rowptr": [0], "idx": [], "kptr": [0], "ktask": [],
          "rptr": [0], "rtask": [], "rforget": []}
    hb["lo"] = lo
    LS = _load_repo_module("loss") if chains else None
    stim = [len(rec["task"])]
    round_ptr = [0]
    rounds, nplaced = [], []
    done = 0
    first_run = set(range(2 * P + 1, 3 * P + 1))  # unpacks not yet restricted
    started = False

    def push(kind, t=-1, w=-1, x=math.nan, nbytes=-1, start=math.nan, stop=math.nan, runid=-1):
        for k, v in zip(ev, (kind, t, w, x, nbytes, start, stop, runid)):
            ev[k].append(v)
        hb["ptr"].append(len(hb["task"]))

    run_of = []
    orig_add = S._add_to_processing

    def add_to_processing(self, ts, ws, stimulus_id):
        r = orig_add(self, ts, ws, stimulus_id)
        run_of.append(int(ts.run_id))
        return r

    S._add_to_processing = add_to_processing
    run_of.extend([int(tss[t].run_id) for t in rec["task"]])
    workers = list(s.workers)  # the plugin's worker_for order (SortedDict: index order)
    while True:
        cur = len(rec["task"])
        batch = list(range(done, cur))
        rounds.append(G.snapshot(s, W, widx) + (len(s.queued),))
        nplaced.append(cur - done)
        done = cur
        if not batch:
            break
        for pos in batch:
            t = rec["task"][pos]
            ts = tss[t]
            if ts.state != "processing" or int(ts.run_id) != run_of[pos]:
                continue
            w = widx[ts.processing_on.address]
            if t in transfers and not started:  # the first transfer runs: the shuffle starts
                plugin._ensure_output_tasks_are_non_rootish(spec)
                assert all(d._rootish is False for d in bar.dependents)
                hb["task"].extend(sorted(tidx[d.key] for d in bar.dependents))
                hb["dur"].extend([0.0] * len(bar.dependents))
                push(EV_SHUFFLE_INIT)
                stim.append(0)
                started = True
            if t in first_run:  # an unpack's first run: restrict_task, then Reschedule
                first_run.discard(t)
                j = t - (2 * P + 1)
                wf = widx[_get_worker_for_range_sharding(P, j, workers)]
                plugin._set_restriction(ts, addr[wf])
                push(EV_RESTRICT, t, wf)
                stim.append(0)
                n0 = len(rec["task"])
                s._reschedule(ts.key, addr[w], stimulus_id=f"reschedule-{len(ev['kind'])}")
                push(EV_RESCHEDULE, t, w)
                dumps.append(_dump(s, g, tidx, widx, [x.key for x in tss]))
                stim.append(len(rec["task"]) - n0)
                continue
            sid_ = f"task-finished-{len(ev['kind'])}"
            r, cm, wm = s.stimulus_task_finished(
                ts.key, ts.processing_on.address, sid_, int(ts.run_id), nbytes=int(g["nbytes"][t]), type=None,
                typename="int", metadata=None,
                startstops=[{"action": "compute", "start": float(g["start"][t]), "stop": float(g["stop"][t])}])
            n0 = len(rec["task"])
            s._transitions(r, cm, wm, sid_)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid_)
            stim.append(len(rec["task"]) - n0)
            push(EV_FINISHED, t, w, math.nan, int(g["nbytes"][t]), float(g["start"][t]), float(g["stop"][t]), pos)
        round_ptr.append(len(ev["kind"]))
    assert not first_run and started
    rec["stim"] = stim
    states = np.array([G.STATE_CODES[ts.state] for ts in tss], np.uint8)
    return rec, rounds, nplaced, states, ev, hb, round_ptr


def main_p2p(only):
    """svcp2p_*: the P2P shuffle lifecycle (replay_p2p), resync dumps after each reschedule."""
    cases = {
        "svcp2p_sat1.1": (lambda: G.graphs.shuffle_graph(200, 16, seed=61, live=True), 1.1),
        "svcp2p_satinf": (lambda: G.graphs.shuffle_graph(160, 12, seed=62, live=True), float("inf")),
    }
    for name, (mk, sat) in cases.items():
        if only and name not in only:
            continue
        g = mk()
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        dumps = []
        rec, rounds, nplaced, states, ev, hb, round_ptr = replay_p2p(g, cfg, dumps)
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(ev_kind=np.array(ev["kind"], np.int8), ev_task=np.array(ev["task"], np.int32),
                 ev_worker=np.array(ev["worker"], np.int32), ev_x=np.array(ev["x"], np.float64),
                 ev_nbytes=np.array(ev["nbytes"], np.int64), ev_start=np.array(ev["start"]),
                 ev_stop=np.array(ev["stop"]), ev_runid=np.array(ev["runid"], np.int64),
                 hb_ptr=np.array(hb["ptr"], np.int64), hb_task=np.array(hb["task"], np.int32),
                 hb_dur=np.array(hb["dur"], np.float64), ev_round_ptr=np.array(round_ptr, np.int64))
        z.update(_pack_dumps(dumps))
        np.savez_compressed(path, **z)
        cnt = np.bincount(np.array(ev["kind"]), minlength=13).tolist()
        print(f"{name}: {len(ev['kind'])} events (by kind {cnt}), {len(dumps)} resyncs, {len(rec['task'])} placements, "
              f"{os.path.getsize(path) / 1e3:.0f} kB")


def main_events(only):
    cases = {
        # every kind, queuing on, random durations, 1-4 threads
        "svcev_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=41, n_inner_prefixes=3,
                                                            random_durations=True, nthreads="random"), 1.1, 41, 0.08),
        # queuing off (root-ish co-assignment reads idle / running)
        "svcev_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 32, seed=42), float("inf"), 42, 0.08),
        # a denser event mix on a smaller graph
        "svcev_dense_sat1.0": (lambda: G.graphs.random_dag(1500, 24, seed=43, n_inner_prefixes=2,
                                                            random_durations=True), 1.0, 43, 0.3),
    }
    for name, (mk, sat, seed, p_event) in cases.items():
        if only and name not in only:
            continue
        g = mk()
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        rec, rounds, nplaced, states, ev, hb, round_ptr = replay_events(g, cfg, seed, p_event)
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(ev_kind=np.array(ev["kind"], np.int8), ev_task=np.array(ev["task"], np.int32),
                 ev_worker=np.array(ev["worker"], np.int32), ev_x=np.array(ev["x"], np.float64),
                 ev_nbytes=np.array(ev["nbytes"], np.int64), ev_start=np.array(ev["start"]),
                 ev_stop=np.array(ev["stop"]), ev_runid=np.array(ev["runid"], np.int64),
                 hb_ptr=np.array(hb["ptr"], np.int64), hb_task=np.array(hb["task"], np.int32),
                 hb_dur=np.array(hb["dur"], np.float64), ev_round_ptr=np.array(round_ptr, np.int64))
        z.update(_tm_arrays(ev["tm"]))
        np.savez_compressed(path, **z)
        cnt = np.bincount(np.array(ev["kind"]), minlength=8).tolist()
        print(f"{name}: {len(ev['kind'])} events (by kind {cnt}), {len(rec['task'])} placements")


def loss_allowed_failures(name):
    """Scheduler.allowed_failures of a loss stream (tests/ext_driver.py sets the same)."""
    return 0 if name.startswith("svcwl_killed0_") else 1 if name.startswith("svcwl_killed_") else 3


def main_resync(only):
    """svcrs_*: the event streams plus the stimuli the engine does not model (worker removal,
    rescheduling, client releases), each followed by the scheduler's state (resync rows)."""
    kinds = (1, 2, 3, 4, 5, 6, 7, 8, 9, 10)
    cases = {
        "svcrs_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=51, n_inner_prefixes=3,
                                                            random_durations=True, nthreads="random"), 1.1, 51, 0.08),
        "svcrs_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=52), float("inf"), 52, 0.08),
        # drained workers retiring among the other events, no resync stimulus
        "svcrt_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=53, n_inner_prefixes=3,
                                                            random_durations=True, nthreads="random"), 1.1, 53, 0.1),
        "svcrt_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=54), float("inf"), 54, 0.1),
        # workers lost with processing tasks / sole replicas, decided by the engine
        "svcwl_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=55, n_inner_prefixes=3,
                                                            random_durations=True, nthreads="random"), 1.1, 55, 0.1),
        "svcwl_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=56), float("inf"), 56, 0.1),
        # ... whose lost results recompute released dependencies (recompute chains)
        "svcwl_chain_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=57, n_inner_prefixes=3,
                                                                  random_durations=True, nthreads="random"), 1.1, 57, 0.1),
        "svcwl_chain_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=58), float("inf"), 58, 0.1),
        # ... and tasks out of retries (allowed_failures 1: a task on its second lost worker errs)
        "svcwl_killed_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=59, n_inner_prefixes=3,
                                                                   random_durations=True, nthreads="random"), 1.1, 59, 0.12),
        "svcwl_killed_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=60), float("inf"), 60, 0.12),
        # clients release results in memory (forgotten / released, the dependencies they forget)
        "svcrel_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=63, n_inner_prefixes=3,
                                                             random_durations=True, nthreads="random"), 1.1, 63, 0.12),
        "svcrel_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=64), float("inf"), 64, 0.12),
        # clients release wanted tasks in any state: cancelled work (waiting, processing, queued,
        # no-worker) and results, with what the transitions release and forget in turn
        "svccan_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=65, n_inner_prefixes=3,
                                                             random_durations=True, nthreads="random"), 1.1, 65, 0.12),
        "svccan_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=66), float("inf"), 66, 0.12),
        # task-erred reports that do not err: retries and stale runs, re-placed by the engine
        "svcretry_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=67, n_inner_prefixes=3,
                                                               random_durations=True, nthreads="random"), 1.1, 67, 0.1),
        "svcretry_c2mini_satinf": (lambda: G.graphs.random_dag(2500, 40, seed=68), float("inf"), 68, 0.1),
        # allowed_failures 0: every processing task of a lost worker errs
        "svcwl_killed0_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 48, seed=61, n_inner_prefixes=3,
                                                                    random_durations=True, nthreads="random"), 1.1, 61, 0.12),
    }
    for name, (mk, sat, seed, p_event) in cases.items():
        if only and name not in only:
            continue
        g = mk()
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        dumps = []
        kinds_ = ((1, 2, 3, 4, 5, 6, 7, EV_RETIRE, EV_RETIRE, EV_PAUSE) if name.startswith("svcrt_") else
                  (1, 2, 3, 4, 5, 6, 7, EV_LOSE_WORKER, EV_LOSE_WORKER, EV_RESUME) if name.startswith("svcwl_") else
                  (1, 2, 3, 4, 5, 6, 7, EV_RELEASE_KEYS, EV_RELEASE_KEYS) if name.startswith(("svcrel_", "svccan_"))
                  else (1, 2, 3, 4, 5, 6, 7, EV_ERRED_RETRY, EV_ERRED_RETRY) if name.startswith("svcretry_")
                  else kinds)
        rec, rounds, nplaced, states, ev, hb, round_ptr = replay_events(
            g, cfg, seed, p_event, kinds_, dumps=dumps, chains=name.startswith(("svcwl_chain_", "svcwl_killed")),
            allowed_failures=loss_allowed_failures(name), release_memory=name.startswith("svcrel_"),
            release_cancel=name.startswith("svccan_"))
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(ev_kind=np.array(ev["kind"], np.int8), ev_task=np.array(ev["task"], np.int32),
                 ev_worker=np.array(ev["worker"], np.int32), ev_x=np.array(ev["x"], np.float64),
                 ev_nbytes=np.array(ev["nbytes"], np.int64), ev_start=np.array(ev["start"]),
                 ev_stop=np.array(ev["stop"]), ev_runid=np.array(ev["runid"], np.int64),
                 hb_ptr=np.array(hb["ptr"], np.int64), hb_task=np.array(hb["task"], np.int32),
                 hb_dur=np.array(hb["dur"], np.float64), ev_round_ptr=np.array(round_ptr, np.int64))
        if dumps:
            z.update(_pack_dumps(dumps))
        lo = hb["lo"]
        if lo["rtask"]:
            z.update(rk_evptr=np.array(lo["rptr"], np.int64), rk_task=np.array(lo["rtask"], np.int32),
                     rk_forget=np.array(lo["rforget"], np.uint8))
        if lo["task"] or lo["ktask"]:
            z.update(lo_evptr=np.array(lo["evptr"], np.int64), lo_task=np.array(lo["task"], np.int32),
                     lo_kind=np.array(lo["kind"], np.int8), lo_rowptr=np.array(lo["rowptr"], np.int64),
                     lo_idx=np.array(lo["idx"], np.int32), lo_kptr=np.array(lo["kptr"], np.int64),
                     lo_ktask=np.array(lo["ktask"], np.int32))
        np.savez_compressed(path, **z)
        if hb.get("dbg"):
            np.save(os.path.join(HERE, f"_dbg_{name}.npy"), np.stack(hb["dbg"]))
        cnt = np.bincount(np.array(ev["kind"]), minlength=16).tolist()
        print(f"{name}: {len(ev['kind'])} events (by kind {cnt}), {len(dumps)} resyncs, {len(rec['task'])} placements, "
              f"{len(lo['task'])} order rows, {len(lo['ktask'])} killed, {os.path.getsize(path) / 1e3:.0f} kB")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "resync":
        return main_resync(set(sys.argv[2:]))
    if len(sys.argv) > 1 and sys.argv[1] == "p2p":
        return main_p2p(set(sys.argv[2:]))
    if len(sys.argv) > 1 and sys.argv[1] == "add-workers":
        return main_add_workers(set(sys.argv[2:]))
    if len(sys.argv) > 1 and sys.argv[1] == "second-graph":
        return main_second_graph(set(sys.argv[2:]))
    if len(sys.argv) > 1 and sys.argv[1] == "events":
        return main_events(set(sys.argv[2:]))
    if len(sys.argv) > 1 and sys.argv[1] == "prefixes":
        return main_prefixes(set(sys.argv[2:]))
    cases = {
        "svc_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 64, seed=15, n_inner_prefixes=3,
                                                          random_durations=True, nthreads="random"), 1.1, 1, 0.0),
        "svc_c2mini_satinf": (lambda: G.graphs.random_dag(2000, 32, seed=16), float("inf"), 2, 0.0),
        "svc_steal_c2var_sat1.1": (lambda: G.graphs.random_dag(3000, 64, seed=17, n_inner_prefixes=3,
                                                                random_durations=True, nthreads="random"), 1.1, 3, 0.05),
        "svc_steal_c2mini_satinf": (lambda: G.graphs.random_dag(2000, 32, seed=18), float("inf"), 4, 0.05),
    }
    only = set(sys.argv[1:])
    for name, (mk, sat, seed, p_steal) in cases.items():
        if only and name not in only:
            continue
        g = mk()
        G.graphs.check_graph(g)
        dask.config.set({"distributed.scheduler.worker-saturation": sat})
        cfg = G.config_dict(sat)
        rec, rounds, nplaced, states, msgs, round_ptr, steals = replay_service(g, cfg, seed, p_steal=p_steal)
        G.save(name, g, cfg, rec, rounds, nplaced, states, 0.0)
        path = os.path.join(HERE, f"{name}.npz")
        z = dict(np.load(path, allow_pickle=False))
        z.update(msg_task=np.array(msgs["task"], np.int32), msg_worker=np.array(msgs["worker"], np.int32),
                 msg_runid=np.array(msgs["run_id"], np.int64), msg_nbytes=np.array(msgs["nbytes"], np.int64),
                 msg_start=np.array(msgs["start"]), msg_stop=np.array(msgs["stop"]),
                 msg_status=np.array(msgs["status"], np.int8), msg_round_ptr=np.array(round_ptr, np.int64))
        if p_steal:
            z.update(steal_msg=np.array(steals["msg"], np.int64), steal_task=np.array(steals["task"], np.int32),
                     steal_thief=np.array(steals["thief"], np.int32))
        np.savez_compressed(path, **z)
        cnt = np.bincount(np.array(msgs["status"]), minlength=5)
        print(f"{name}: {len(msgs['task'])} messages, statuses {cnt.tolist()}, {len(steals['task'])} steals")


if __name__ == "__main__":
    main()
