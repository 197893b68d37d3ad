"""Drives the drop-in extension (``distributed_amd/ext.py``) inside the *reference*
scheduler state (python3.9 + ``tests/golden/_refshim.py``; build container only — the
reference does not travel to the GPU box). Called by ``tests/test_ext.py``.

For each golden fixture: the reference ``SchedulerState`` of ``gen_golden.build_state``
(canonical tie-break instrumentation) gets a ``GPUPlacementExtension`` whose engine is a
stand-in serving the fixture's own placement log, stimulus by stimulus
(``stim_nplaced``): the engine outputs are fixture data, made by the reference itself.
Then the replay protocol runs through the scheduler's real entry points:

* ``update_graph``: the extension's ``SchedulerPlugin.update_graph`` hook, then the
  scheduler's transitions (``scheduler.py:4641-4653``);
* every completion through ``stream_handlers["task-finished"]`` -> the extension ->
  ``Scheduler.handle_task_finished`` (``:5783-5797``).

Checks: the graph the extension uploads equals the fixture graph (the TaskState -> CSR
conversion), every placement the scheduler made came from the engine in the engine's
order, ``validate=True`` re-derives each one with the reference's ``decide_worker*`` and
finds it equal, and the placement records equal the fixture's. ``--diverge`` swaps two
decisions of one stimulus: the extension must detect it, hand placement back to the
scheduler's own decide_worker, and the records must still equal the fixture's.
Prints one JSON line per fixture.
"""
from __future__ import annotations

import json
import os
import sys
import time as _time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
if os.environ.get("PYTHONHASHSEED") != "0":
    import subprocess

    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, PYTHONHASHSEED="0")))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import gen_golden as G  # noqa: E402  (shim + reference)

import dask  # noqa: E402
import numpy as np  # noqa: E402

from distributed.scheduler import Scheduler  # noqa: E402
from distributed_amd.ext import GPUPlacementExtension  # noqa: E402
from oracle.oracle import load_fixture  # noqa: E402


class FixtureEngine:
    """The engine interface ext.py uses, serving a reference fixture's placement log."""

    def __init__(self, exp, fixture_keys):
        self.exp = exp
        self.fkeys = fixture_keys
        self.stim = exp["stim_nplaced"].tolist()
        self.n = 0
        self.k = 0
        self.ext = None
        self.graph = None
        self.diverge = None  # placement index whose decision is swapped with the next one
        self.graphs = []
        self.calls_tf = 0  # dgp_tasks_finished calls the extension made
        self._posted = None
        self.t_window = 0.0
        self.windows = []
        self.joins = []  # add_worker calls: (nthreads, running, position)

    def load(self, g, config, results=True):
        self.graph, self.config = g, config
        self.deps = []  # engine index -> its dependencies' engine indices (CSR order)
        self._append_deps(g)
        self.who, self.nb = {}, {}  # replicas / reported sizes as the engine holds them

    def _append_deps(self, g):
        base = len(self.deps)
        dp, di = np.asarray(g["dep_ptr"]), np.asarray(g["dep_idx"])
        for i in range(len(dp) - 1):
            self.deps.append([int(d) + base if d >= 0 else -1 - int(d) for d in di[dp[i]:dp[i + 1]]])

    def set_resident(self, on=True):  # the real engine's launch mode: nothing to serve here
        self.resident = bool(on)

    def set_task_messages(self, on=True):  # the real engine's mailbox message fields: task_messages below
        self.task_msgs = bool(on)

    def update_graph(self):
        self.n, self.k = self.stim[0], 1

    def tasks_finished(self, task, worker, run_id, nbytes=None, start=None, stop=None):
        return self._finished(task, worker, run_id, nbytes, start, stop)

    def tasks_finished_post(self, *args):  # dgp_tasks_finished_post: answered at the wait
        assert self._posted is None, "a batch posted twice"
        self._posted = args
        self._t_post = _time.perf_counter()

    def tasks_finished_wait(self):
        # the host time between post and wait: the window the device's answer overlaps
        dt_ = _time.perf_counter() - self._t_post
        self.t_window += dt_
        self.windows.append(dt_)
        args, self._posted = self._posted, None
        assert args is not None, "no batch posted"
        return self._finished(*args)

    def _finished(self, task, worker, run_id, nbytes=None, start=None, stop=None):
        self.calls_tf += 1
        n0 = self.n
        for i, t in enumerate(task):  # genuine completions only in this protocol
            self.n += self.stim[self.k]
            self.k += 1
            self.who[int(t)] = {int(worker[i])}
            self.nb[int(t)] = -1 if nbytes is None else int(nbytes[i])
        return np.zeros(len(task), np.int8), self.n - n0

    def task_messages(self, offset, count):
        """dgp_task_messages' arrays from the replicas this stand-in tracked (the placement
        log's tasks from placements(); holders ascending)."""
        tasks = self.placements(offset, count)["pl_task"].tolist()
        ptr, dt, dn, hp, hi = [0], [], [], [0], []
        for t in tasks:
            for d in self.deps[t]:
                dt.append(d)
                dn.append(self.nb.get(d, -1))
                hi.extend(sorted(self.who.get(d, ())))
                hp.append(len(hi))
            ptr.append(len(dt))
        return dict(dep_ptr=np.array(ptr, np.int64), dep_task=np.array(dt, np.int32), dep_nbytes=np.array(dn, np.int64),
                    holder_ptr=np.array(hp, np.int64), holder_idx=np.array(hi, np.int32))

    def answer(self, offset, count, messages=True):  # PlacementEngine.answer from the two calls it fuses
        pl = self.placements(offset, count)
        batch = None
        if messages:
            m = self.task_messages(offset, count)
            batch = tuple(m[k].tolist() for k in ("dep_ptr", "dep_task", "dep_nbytes", "holder_ptr", "holder_idx"))
        return pl["pl_task"].tolist(), pl["pl_worker"].tolist(), batch

    def num_placements(self):
        assert self._posted is None, "num_placements while a batch is posted"
        return self.n

    def placements(self, offset=0, count=None, columns=None):
        assert self._posted is None, "placements while a batch is posted"
        sl = slice(offset, offset + count)
        idx = self.ext.task_index
        task = np.array([idx[self.fkeys[t]] for t in self.exp["pl_task"][sl]], np.int32)
        if self.diverge is not None and offset <= self.diverge < offset + count - 1:
            j = self.diverge - offset  # two decisions of one stimulus swapped
            task[j], task[j + 1] = task[j + 1], task[j]
        return {"pl_task": task, "pl_worker": self.exp["pl_worker"][sl]}

    def add_graph(self, g, defer=False):  # a later graph (the fixture's per-event placement counts)
        self.graphs.append(g)
        self._append_deps(g)
        if defer or (np.asarray(g["dep_idx"]) < 0).any():  # appended, the scheduler's stimulus, then sync()
            return 0
        return self.add_worker(0)

    def add_worker(self, nthreads, running=True, position=None):  # a join (the fixture's per-event placement counts)
        assert self._posted is None, "add_worker while a batch is posted"
        self.joins.append((int(nthreads), bool(running), position))
        if position is not None:  # dgp_add_worker_at: every later worker index moves up by one
            self.who = {t: {w + (w >= position) for w in ws} for t, ws in self.who.items()}
        k = self.stim[self.k]
        self.n += k
        self.k += 1
        return k

    def close(self):
        pass


def check_upload(g_up, keys_up, g_fx, fkeys):
    """The extension's TaskState -> CSR conversion against the fixture graph (graphs.py)."""
    pos = {k: i for i, k in enumerate(fkeys)}
    perm = np.array([pos[k] for k in keys_up])  # upload index -> fixture index
    assert len(perm) == g_fx["n_tasks"]
    for i, f in enumerate(perm):
        up = sorted(fkeys[perm[d]] for d in g_up["dep_idx"][g_up["dep_ptr"][i]:g_up["dep_ptr"][i + 1]])
        fx = sorted(fkeys[d] for d in g_fx["dep_idx"][g_fx["dep_ptr"][f]:g_fx["dep_ptr"][f + 1]])
        assert up == fx, (keys_up[i], up, fx)
    pn_up = np.array(g_up["prefix_names"])[g_up["prefix_id"]]
    pn_fx = np.array(g_fx["prefix_names"])[g_fx["prefix_id"][perm]]
    assert (pn_up == pn_fx).all()
    gn_up = np.array(g_up["group_names"])[g_up["group_id"]]
    gn_fx = np.array(g_fx["group_names"])[g_fx["group_id"][perm]]
    assert (gn_up == gn_fx).all()
    assert np.array_equal(g_up["wanted"], g_fx["wanted"][perm])
    assert np.array_equal(g_up["rootish_override"], g_fx["rootish_override"][perm])
    assert np.array_equal(g_up["nthreads"], g_fx["nthreads"])
    # restrictions: TaskState.worker_restrictions -> valid_workers -> indices (f1)
    if "restr_flags" in g_fx:
        assert np.array_equal(g_up["restr_flags"], g_fx["restr_flags"][perm])
        for i, f in enumerate(perm):
            up = g_up["restr_idx"][g_up["restr_ptr"][i]:g_up["restr_ptr"][i + 1]].tolist()
            fx = g_fx["restr_idx"][g_fx["restr_ptr"][f]:g_fx["restr_ptr"][f + 1]].tolist()
            assert up == fx, (keys_up[i], up, fx)
    else:
        assert "restr_flags" not in g_up
    # priority rank: ascending fixture priority
    assert np.array_equal(np.argsort(g_fx["prio"][perm], kind="stable"), np.arange(len(perm)))
    # the engine's prefix table = TaskPrefix.duration_average at upload
    pd_fx = dict(zip(g_fx["prefix_names"], g_fx["prefix_default_dur"]))
    assert all(pd_fx[n] == d for n, d in zip(g_up["prefix_names"], g_up["prefix_default_dur"]))


def check_messages(g, exp, sent, fkeys):
    """The host-model compute-task fields (tests/msg_model.py) against the
    reference's own messages: key, priority, who_has, nbytes, run_id order."""
    from msg_model import compute_task_batch, render_messages

    n = len(exp["pl_task"])
    assert len(sent) == n, (len(sent), n)
    batch = compute_task_batch(g, exp["pl_task"], exp["pl_worker"], 0, n, g["nbytes"])
    addrs = [f"tcp://w{i:05d}:1" for i in range(len(g["nthreads"]))]
    mine = render_messages(batch, fkeys, addrs, lambda t: (0, 1, int(g["prio"][t])), lambda t: 0.0)
    for a, b in zip(mine, sent):
        assert a["key"] == b["key"] and a["priority"] == b["priority"], (a["key"], b["key"])
        assert {k: sorted(v) for k, v in a["who_has"].items()} == {k: sorted(v) for k, v in b["who_has"].items()}, a["key"]
        assert a["nbytes"] == b["nbytes"], a["key"]
    assert [m["run_id"] for m in sent] == sorted(m["run_id"] for m in sent)


class FakeComm:
    """A worker's batched stream as ``Server.handle_stream`` reads it: each ``read()`` returns
    one batch (list of messages), then the comm closes."""

    peer_address = "tcp://fake:0"

    def __init__(self, batches):
        self.batches = list(batches)
        self.closed_ = False

    async def read(self):
        from distributed.comm.core import CommClosedError

        if not self.batches:
            raise CommClosedError("done")
        return self.batches.pop(0)

    async def close(self):
        self.closed_ = True

    def closed(self):
        return self.closed_


def run(name, diverge=False, stream=False, plain=False, validate=True):
    """One fixture's replay protocol through the extension (or, ``plain``, through the
    reference handlers alone, for timing). ``stream``: each round's messages arrive as
    comm batches (consecutive messages of one worker per ``comm.read``) through the
    extension's ``handle_stream``, one engine call per batch."""
    import asyncio
    import time as _time

    g, cfg, exp, meta = load_fixture(os.path.join(HERE, "golden", name))
    g["keys"] = None
    sat = cfg["saturation"]
    sat = float("inf") if sat == "inf" else float(sat)
    dask.config.set({"distributed.scheduler.worker-saturation": sat})
    cfg = dict(cfg, saturation=sat)
    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    S = type(s)
    S.stimulus_task_finished = Scheduler.stimulus_task_finished
    S.handle_task_finished = Scheduler.handle_task_finished
    S.validate_key = lambda self, key, ts=None: None
    S.send_all = lambda self, client_msgs, worker_msgs: None
    sent = []  # every compute-task message the reference built (_task_to_msg :3421-3450)
    orig_msg = S._task_to_msg

    def task_to_msg(self, ts, duration=-1):
        m = orig_msg(self, ts, duration)
        sent.append(m)
        return m

    S._task_to_msg = task_to_msg
    fkeys = [ts.key for ts in tss]
    if plain:  # the unmodified reference: its own decisions, its own handler
        s.stream_handlers = {"task-finished": lambda **kw: Scheduler.handle_task_finished(s, **kw)}
        if plain == "plugin":  # a SchedulerPlugin registered, as WorkStealing is in production
            from distributed.diagnostics.plugin import SchedulerPlugin

            s.plugins = {"noop": SchedulerPlugin()}
        recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
        s._transitions(recs, {}, {}, "update-graph")
        done, n_msgs, t_msgs, c_msgs = 0, 0, 0.0, 0.0
        while True:
            cur = len(rec["task"])
            batch = rec["task"][done:cur]
            done = cur
            if not batch:
                break
            t0, c0 = _time.perf_counter(), _time.process_time()
            for t in batch:
                ts = tss[t]
                s.stream_handlers["task-finished"](
                    key=ts.key, worker=ts.processing_on.address, stimulus_id=f"tf-{t}", run_id=ts.run_id,
                    nbytes=int(g["nbytes"][t]), type=None, typename="int", metadata=None,
                    startstops=[{"action": "compute", "start": float(g["start"][t]), "stop": float(g["stop"][t])}])
            t_msgs += _time.perf_counter() - t0
            c_msgs += _time.process_time() - c0
            n_msgs += len(batch)
        assert rec["task"] == exp["pl_task"].tolist()
        return dict(fixture=name, mode="plain" if plain is True else "plain+plugin", messages=n_msgs,
                    us_per_message=round(1e6 * t_msgs / n_msgs, 2),
                    cpu_us_per_message=round(1e6 * c_msgs / n_msgs, 2))
    eng = FixtureEngine(exp, fkeys)
    if diverge:  # first stimulus after update_graph with two or more placements
        stim = exp["stim_nplaced"]
        pos = np.cumsum(stim) - stim
        k = next(i for i in range(1, len(stim)) if stim[i] >= 2 and exp["pl_task"][pos[i]] != exp["pl_task"][pos[i] + 1])
        eng.diverge = int(pos[k])
    S._task_to_msg = orig_msg  # the extension wraps the instance's: every message recorded below
    eng.t_engine = eng.c_engine = 0.0
    for nm_ in ("tasks_finished", "tasks_finished_post", "tasks_finished_wait", "placements", "task_messages",
                "num_placements"):
        def timed(*a, _f=getattr(eng, nm_), **k):
            t0_, c0_ = _time.perf_counter(), _time.process_time()
            try:
                return _f(*a, **k)
            finally:
                eng.t_engine += _time.perf_counter() - t0_
                eng.c_engine += _time.process_time() - c0_
        setattr(eng, nm_, timed)
    ext = GPUPlacementExtension(s, engine_factory=lambda: eng, validate=validate)
    ext.overlap = "--nooverlap" not in sys.argv
    eng.ext = ext
    s.stream_handlers = {}
    ext._install()  # with the stream handler table in place
    ext_msg = s._task_to_msg

    def record_msg(ts, duration=-1):
        m = ext_msg(ts, duration)
        sent.append(m)
        return m

    s._task_to_msg = record_msg
    # Scheduler._create_taskstate_from_graph's tail (:4600-4653): plugin hook, then transitions
    priority = {ts.key: ts.priority for ts in tss}
    recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                     priority=priority, dependencies={})
    assert ext.active, ext.reason
    check_upload(eng.graph, ext.keys, g, fkeys)
    s._transitions(recs, {}, {}, "update-graph")
    done = 0
    n_msgs = 0
    n_reads = 0
    t_msgs = c_msgs = 0.0
    calls0 = ext.stats.get("messages", 0)
    while True:
        cur = len(rec["task"])
        batch = rec["task"][done:cur]
        done = cur
        if not batch:
            break

        def msg(t):
            ts = tss[t]
            return dict(key=ts.key, stimulus_id=f"tf-{t}", run_id=ts.run_id, nbytes=int(g["nbytes"][t]), type=None,
                        typename="int", metadata=None,
                        startstops=[{"action": "compute", "start": float(g["start"][t]), "stop": float(g["stop"][t])}])
        t0, c0 = _time.perf_counter(), _time.process_time()
        if stream:  # one comm.read per run of consecutive messages from one worker
            runs = []
            for t in batch:
                w = tss[t].processing_on.address
                if runs and runs[-1][0] == w:
                    runs[-1][1].append(t)
                else:
                    runs.append((w, [t]))
            for w, ts_ in runs:  # each worker's comm delivers its batch; the handler reads it
                asyncio.run(ext.handle_stream(FakeComm([[dict(msg(t), op="task-finished") for t in ts_]]),
                                              extra={"worker": w}))
                n_reads += 1
        else:
            for t in batch:
                s.stream_handlers["task-finished"](worker=tss[t].processing_on.address, **msg(t))
        t_msgs += _time.perf_counter() - t0
        c_msgs += _time.process_time() - c0
        n_msgs += len(batch)
    ext._end_of_stimulus("end of replay")
    assert ext.active != diverge, ext.reason  # a divergence hands placement back to the scheduler
    n = len(exp["pl_task"])
    assert rec["task"] == exp["pl_task"].tolist()
    assert rec["worker"] == exp["pl_worker"].tolist()
    assert rec["comm"] == exp["pl_comm"].tolist()
    assert np.array_equal(np.array(rec["start"]).view(np.int64), exp["pl_start"].view(np.int64))
    assert rec["wsnbytes"] == exp["pl_wsnbytes"].tolist()
    if not diverge:
        assert ext.stats["device_decisions"] == n, (ext.stats, n)
        # every compute-task message built from the engine's batch (dgp_task_messages)
        assert ext.n_engine_messages == n, (ext.n_engine_messages, n)
        check_messages(g, exp, sent, fkeys)
    return dict(fixture=name, placements=n, messages=n_msgs, device_decisions=ext.stats["device_decisions"],
                engine_messages=ext.n_engine_messages,
                # the extension and the reference handler without the stand-in engine's own time
                # (on the box the engine call replaces it: bench.py service leg)
                us_per_message_host=round(1e6 * (t_msgs - eng.t_engine) / max(n_msgs, 1), 2),
                cpu_us_per_message_host=round(1e6 * (c_msgs - eng.c_engine) / max(n_msgs, 1), 2),
                # between the post and the first decision: the device answers meanwhile
                us_overlap_window=round(1e6 * eng.t_window / max(eng.calls_tf, 1), 2),
                us_overlap_window_p10_p50=[round(1e6 * float(np.percentile(eng.windows, q)), 1) for q in (10, 50)]
                if eng.windows else None,
                device_queued=ext.stats["device_queued"], device_no_worker=ext.stats["device_no_worker"],
                active=ext.active, reason=ext.reason, engine_calls=eng.calls_tf, reads=n_reads,
                us_per_message=round(1e6 * t_msgs / max(n_msgs, 1), 2), mode="stream" if stream else "handler")


def run_ab(name):
    """Timing A/B of the drop-in: the reference (its own handler, a SchedulerPlugin
    registered) and the extension (overlapped engine call; the stand-in engine's time
    subtracted) on two independent states of the same fixture in ONE process, fed the same
    task-finished messages alternately (which side goes first alternates too). Each message's
    handler time is taken on both sides under the same machine conditions, so the per-message
    difference cancels what other tenants of the machine do; reported with its 95 % interval."""
    from distributed.diagnostics.plugin import SchedulerPlugin

    g, cfg, exp, meta = load_fixture(os.path.join(HERE, "golden", name))
    g["keys"] = None
    sat = cfg["saturation"]
    sat = float("inf") if sat == "inf" else float(sat)
    dask.config.set({"distributed.scheduler.worker-saturation": sat})
    cfg = dict(cfg, saturation=sat)
    sides = {}
    for mode in ("reference", "extension"):
        s, tss, widx, rec, tidx = G.build_state(g, cfg)  # a class of its own per state
        S = type(s)
        S.stimulus_task_finished = Scheduler.stimulus_task_finished
        S.handle_task_finished = Scheduler.handle_task_finished
        S.validate_key = lambda self, key, ts=None: None
        S.send_all = lambda self, client_msgs, worker_msgs: None
        recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
        eng = None
        if mode == "reference":
            s.plugins = {"noop": SchedulerPlugin()}
            handler = (lambda _s: lambda **kw: Scheduler.handle_task_finished(_s, **kw))(s)
        else:
            eng = FixtureEngine(exp, [ts.key for ts in tss])
            eng.t_engine, eng.n_timed, depth = 0.0, 0, [0]
            # the stand-in's time leaves the extension's: every outermost call into it is
            # timed (the real engine's Python wrappers and device time are bench.py's
            # service.per_message_overlap_ext.exposed_us_per_call instead)
            for nm_ in ("tasks_finished", "tasks_finished_post", "tasks_finished_wait", "answer", "placements",
                        "task_messages", "num_placements"):
                def timed(*a, _f=getattr(eng, nm_), **k):
                    if depth[0]:
                        return _f(*a, **k)
                    depth[0] = 1
                    t0_ = _time.perf_counter()
                    try:
                        return _f(*a, **k)
                    finally:
                        eng.t_engine += _time.perf_counter() - t0_
                        eng.n_timed += 1
                        depth[0] = 0
                setattr(eng, nm_, timed)

            def _noop():
                pass

            def _timed_noop(*a, _f=_noop, **k):  # the wrapper's own cost, taken off per timed call
                if depth[0]:
                    return _f(*a, **k)
                depth[0] = 1
                t0_ = _time.perf_counter()
                try:
                    return _f(*a, **k)
                finally:
                    eng.t_engine += _time.perf_counter() - t0_
                    eng.n_timed += 1
                    depth[0] = 0
            t_cal = _time.perf_counter()
            for _ in range(200_000):
                _timed_noop()
            eng.wrap_s = (_time.perf_counter() - t_cal) / 200_000
            eng.t_engine, eng.n_timed = 0.0, 0
            ext = GPUPlacementExtension(s, engine_factory=lambda: eng, validate=False)
            eng.ext = ext
            ext.overlap = os.environ.get("AB_OVERLAP", "1") == "1"  # knobs for attributing the difference
            ext.engine_messages = os.environ.get("AB_MESSAGES", "1") == "1"
            s.stream_handlers = {}
            ext._install()
            priority = {ts.key: ts.priority for ts in tss}
            ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                             priority=priority, dependencies={})
            assert ext.active, ext.reason
            handler = s.stream_handlers["task-finished"]
        s._transitions(recs, {}, {}, "update-graph")
        sides[mode] = (tss, rec, handler, eng)
    rec0 = sides["reference"][1]
    diffs, tot = [], {"reference": 0.0, "extension": 0.0}
    import gc

    profs = {}
    if os.environ.get("AB_PROFILE"):  # one cProfile per side: call counts and times side by side
        import cProfile

        profs = {"reference": cProfile.Profile(), "extension": cProfile.Profile()}
    gc.collect()
    if os.environ.get("AB_GC") == "freeze":  # the states built above leave the collector's scans
        gc.freeze()
    elif os.environ.get("AB_GC") == "off":
        gc.disable()
    done, i = 0, 0
    while True:
        cur = len(rec0["task"])
        batch = rec0["task"][done:cur]
        done = cur
        if not batch:
            break
        for t in batch:
            dt = {}
            for mode in (("reference", "extension") if i % 2 == 0 else ("extension", "reference")):
                tss, rec, handler, eng = sides[mode]
                ts = tss[t]
                kw = dict(key=ts.key, worker=ts.processing_on.address, stimulus_id=f"tf-{t}", run_id=ts.run_id,
                          nbytes=int(g["nbytes"][t]), type=None, typename="int", metadata=None,
                          startstops=[{"action": "compute", "start": float(g["start"][t]),
                                       "stop": float(g["stop"][t])}])
                e0, n0 = (eng.t_engine, eng.n_timed) if eng else (0.0, 0)
                prof = profs.get(mode)
                if prof:
                    prof.enable()
                t0 = _time.perf_counter()
                handler(**kw)
                d = _time.perf_counter() - t0
                if prof:
                    prof.disable()
                if eng:
                    d -= eng.t_engine - e0 + (eng.n_timed - n0) * eng.wrap_s
                dt[mode] = d
                tot[mode] += d
            diffs.append(dt["extension"] - dt["reference"])
            i += 1
    ext = sides["extension"][3].ext
    ext._end_of_stimulus("end of replay")
    for mode in sides:
        assert sides[mode][1]["task"] == exp["pl_task"].tolist(), mode
    assert ext.active and ext.stats["device_decisions"] == len(exp["pl_task"]), (ext.reason, ext.stats)
    assert ext.n_engine_messages == (len(exp["pl_task"]) if ext.engine_messages else 0)
    for mode, prof in profs.items():
        prof.dump_stats(os.path.join(os.environ["AB_PROFILE"], f"ab_{mode}.prof"))
    d = np.array(diffs) * 1e6
    half = 1.96 * d.std(ddof=1) / np.sqrt(len(d))
    return dict(fixture=name, mode="ab", messages=i,
                reference_us_per_message=round(1e6 * tot["reference"] / i, 2),
                extension_host_us_per_message=round(1e6 * tot["extension"] / i, 2),
                diff_us_per_message=round(float(d.mean()), 2), diff_ci95_us=round(float(half), 2),
                diff_median_us=round(float(np.median(d)), 2))


def run_joins(name):
    """A ``svcaddw_*`` stream (gen_service.py add-workers): workers join between the
    task-finished messages through the placement-relevant body of ``Scheduler.add_worker``
    (scheduler.py:4370-4420: workers / running / total_nthreads, check_idle_saturated, the
    plugins' add_worker hook, bulk_schedule_unrunnable_after_adding_worker,
    stimulus_queue_slots_maybe_opened); the extension's hook adds the worker to the engine
    and its queue refill decisions are the ones the scheduler then takes. ``svcaddw_order_*``:
    the addresses sort among the known ones (the extension must insert each at its SortedDict
    place, dgp_add_worker_at) and some join paused, resuming later through the scheduler's
    worker-status-change handler."""
    from distributed.core import Status
    from distributed.scheduler import WorkerState

    path = os.path.join(HERE, "golden", name)
    g, cfg, exp, meta = load_fixture(path)
    z = np.load(path, allow_pickle=False)
    g["keys"] = None
    sat = cfg["saturation"]
    sat = float("inf") if sat == "inf" else float(sat)
    dask.config.set({"distributed.scheduler.worker-saturation": sat})
    cfg = dict(cfg, saturation=sat)
    step = int(z["addr_step"]) if "addr_step" in z.files else 0
    s, tss, widx, rec, tidx = G.build_state(g, cfg, (lambda i: f"tcp://w{step * i:07d}:1") if step else None)
    S = type(s)
    S.stimulus_task_finished = Scheduler.stimulus_task_finished
    S.handle_task_finished = Scheduler.handle_task_finished
    S.handle_worker_status_change = Scheduler.handle_worker_status_change
    S.validate_key = lambda self, key, ts=None: None
    S.send_all = lambda self, client_msgs, worker_msgs: None
    s.extensions = {}
    fkeys = [ts.key for ts in tss]
    eng = EventEngine(exp, fkeys)
    eng.joins = []
    ext = GPUPlacementExtension(s, engine_factory=lambda: eng, validate=True)
    eng.ext = ext
    s.stream_handlers = {"worker-status-change": s.handle_worker_status_change}
    ext._install()
    priority = {ts.key: ts.priority for ts in tss}
    recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                     priority=priority, dependencies={})
    assert ext.active, ext.reason
    s._transitions(recs, {}, {}, "update-graph")
    W0 = len(g["nthreads"])
    joins = {}
    n_add = len(z["add_nthreads"])
    addrs = z["add_addr"].tolist() if "add_addr" in z.files else [f"tcp://w{W0 + k:05d}:1" for k in range(n_add)]
    running = z["add_running"].tolist() if "add_running" in z.files else [1] * n_add
    pos = z["add_pos"].tolist() if "add_pos" in z.files else [W0 + k for k in range(n_add)]
    for k, (i, nt) in enumerate(zip(z["add_msg"].tolist(), z["add_nthreads"].tolist())):
        joins.setdefault(i, []).append(k)
    resumes = {}
    for i, w in zip(*((z["res_msg"].tolist(), z["res_worker"].tolist()) if "res_msg" in z.files else ((), ()))):
        resumes.setdefault(i, []).append(w)
    k_join = n_res = 0
    for i, (t, w) in enumerate(zip(z["msg_task"].tolist(), z["msg_worker"].tolist())):
        for k in joins.get(i, ()):
            addr = addrs[k]
            run_ = bool(running[k])
            ws = WorkerState(address=addr, status=Status.running if run_ else Status.paused, pid=0, name=addr,
                             nthreads=int(z["add_nthreads"][k]), memory_limit=0, local_directory="", nanny=None,
                             server_id=addr, scheduler=s)
            s.workers[addr] = ws
            for r_, a in enumerate(s.workers):  # the canonical index is the SortedDict rank
                widx[a] = r_
            assert widx[addr] == pos[k], (addr, widx[addr], pos[k])
            if run_:
                s.running.add(ws)
            s.aliases[addr] = addr
            s.total_nthreads += ws.nthreads
            s.check_idle_saturated(ws)
            ext.add_worker(scheduler=s, worker=addr)
            assert ext.worker_index[addr] == pos[k] and eng.joins[-1] == (ws.nthreads, run_, pos[k]), \
                (ext.worker_index.get(addr), eng.joins[-1], pos[k])
            if run_:
                s.transitions(s.bulk_schedule_unrunnable_after_adding_worker(ws), f"add-{addr}")
                s.stimulus_queue_slots_maybe_opened(stimulus_id=f"add-{addr}")
            k_join += 1
        for w_ in resumes.get(i, ()):  # a paused joiner resumes: the scheduler's own stream handler
            a = next(x for x, r_ in widx.items() if r_ == w_ and x in s.workers)
            s.stream_handlers["worker-status-change"](status="running", worker=a, stimulus_id=f"resume-{a}")
            assert eng.calls[-1] == ("status", w_, 1), eng.calls[-1:]
            n_res += 1
        ts = tss[t]
        assert widx[ts.processing_on.address] == w  # the message's worker index is the SortedDict rank
        s.stream_handlers["task-finished"](
            key=ts.key, worker=ts.processing_on.address, stimulus_id=f"tf-{t}", run_id=ts.run_id,
            nbytes=int(g["nbytes"][t]), type=None, typename="int", metadata=None,
            startstops=[{"action": "compute", "start": float(g["start"][t]), "stop": float(g["stop"][t])}])
    ext._end_of_stimulus("end of stream")
    assert ext.active, ext.reason
    assert k_join == n_add
    assert ext.workers == sorted(s.workers), "the engine's worker order is the SortedDict's"
    n = len(exp["pl_task"])
    assert rec["task"] == exp["pl_task"].tolist()
    assert rec["worker"] == exp["pl_worker"].tolist()
    assert np.array_equal(np.array(rec["start"]).view(np.int64), exp["pl_start"].view(np.int64))
    assert ext.stats["device_decisions"] == n, (ext.stats, n)
    return dict(fixture=name, placements=n, joins=k_join, resumes=n_res, workers_added=ext.stats["workers_added"],
                workers_inserted=ext.stats["workers_inserted"], workers_added_paused=ext.stats["workers_added_paused"],
                device_decisions=ext.stats["device_decisions"], active=ext.active, reason=ext.reason)


def run_second_graph(name, resync=False):
    """A ``svcgraph_*`` stream (gen_service.py second-graph): a second, independent graph is
    submitted mid-stream through the tail of ``_create_taskstate_from_graph``
    (scheduler.py:4600-4653: the plugins' update_graph hook, then the transitions); the
    extension uploads it to the engine (dgp_add_graph) and the scheduler takes the engine's
    decisions for both graphs from then on. ``svcgdep_*``: the second graph depends on earlier
    tasks; the extension appends it, lets the scheduler decide that stimulus and resyncs the
    engine (the rows it sends are the scheduler's state, the fixture's dump)."""
    import operator

    from gen_service import TOKEN2

    path = os.path.join(HERE, "golden", name)
    g, cfg, exp, meta = load_fixture(path)
    z = np.load(path, allow_pickle=False)
    g["keys"] = None
    sat = cfg["saturation"]
    sat = float("inf") if sat == "inf" else float(sat)
    dask.config.set({"distributed.scheduler.worker-saturation": sat})
    cfg = dict(cfg, saturation=sat)
    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    S = type(s)
    S.stimulus_task_finished = Scheduler.stimulus_task_finished
    S.handle_task_finished = Scheduler.handle_task_finished
    S.validate_key = lambda self, key, ts=None: None
    S.send_all = lambda self, client_msgs, worker_msgs: None
    fkeys = [ts.key for ts in tss]
    # the scheduler decides the submission, then a resync (svcgprio_: a user priority above the
    # earlier tasks', the engine takes the merged ranks first)
    dep = name.startswith(("svcgdep_", "svcgrst_", "svcgprio_", "svcgrec_"))
    user_prio = int(z["g2_user_prio"]) if "g2_user_prio" in z.files else 0
    # the engine runs that stimulus (dgp_graph_stimulus) unless ``resync``: the engine of
    # rounds 3-4 without it, the scheduler deciding and a resync after it
    eng = ((EventEngine if resync else GraphStimulusEngine) if dep else FixtureEngine)(exp, fkeys)
    ext = GPUPlacementExtension(s, engine_factory=lambda: eng, validate=True)
    eng.ext = ext
    s.stream_handlers = {}
    ext._install()
    priority = {ts.key: ts.priority for ts in tss}
    recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                     priority=priority, dependencies={})
    assert ext.active, ext.reason
    s._transitions(recs, {}, {}, "update-graph")
    # the second graph, as the generator built it
    g2 = {k[3:]: z[k] for k in z.files if k.startswith("g2_")}
    g2["n_tasks"] = len(g2["prio"])
    g2["prefix_names"] = g["prefix_names"]
    g2["group_names"] = [nm.replace(G.graphs.TOKEN, TOKEN2) for nm in g["group_names"]]
    cs = s.clients["client-0"]
    N1 = g["n_tasks"]
    at = int(z["g2_msg"])
    joins = dict(zip(z["add_msg"].tolist(), z["add_nthreads"].tolist())) if "add_msg" in z.files else {}
    W0 = len(g["nthreads"])
    k_join = 0
    for i, (t, w) in enumerate(zip(z["msg_task"].tolist(), z["msg_worker"].tolist())):
        if i in joins:  # Scheduler.add_worker's placement part (see run_joins)
            from distributed.core import Status
            from distributed.scheduler import WorkerState

            addr = f"tcp://w{W0 + k_join:05d}:1"
            widx[addr] = W0 + k_join
            ws = WorkerState(address=addr, status=Status.running, pid=0, name=addr, nthreads=joins[i],
                             memory_limit=0, local_directory="", nanny=None, server_id=addr, scheduler=s)
            s.workers[addr] = ws
            s.running.add(ws)
            s.aliases[addr] = addr
            s.total_nthreads += ws.nthreads
            s.check_idle_saturated(ws)
            ext.add_worker(scheduler=s, worker=addr)
            s.transitions(s.bulk_schedule_unrunnable_after_adding_worker(ws), f"add-{addr}")
            s.stimulus_queue_slots_maybe_opened(stimulus_id=f"add-{addr}")
            k_join += 1
        if i == at:
            keys2 = G.make_keys(g2)
            new = []
            for k, key in enumerate(keys2):
                ts = s.new_task(key, (operator.add, (), {}), "released")
                tidx[key] = N1 + k
                ts.priority = (-user_prio, 2, int(g2["prio"][k]))
                new.append(ts)
            for k, ts in enumerate(new):
                for d in g2["dep_idx"][g2["dep_ptr"][k]:g2["dep_ptr"][k + 1]]:
                    ts.add_dependency(new[int(d)] if d >= 0 else tss[-1 - int(d)])
                if g2["wanted"][k]:
                    ts.who_wants = {cs}
                    cs.wants_what.add(ts)
                if "restr_flags" in g2 and g2["restr_flags"][k] & 1:  # as the generator set them
                    rp, ri = g2["restr_ptr"], g2["restr_idx"]
                    ts.worker_restrictions = {f"tcp://w{int(x):05d}:1" for x in ri[rp[k]:rp[k + 1]]} | {"tcp://gone:1"}
                    ts.loose_restrictions = bool(g2["restr_flags"][k] & 2)
            eng.fkeys.extend(keys2)
            tss.extend(new)
            prio2 = {ts.key: ts.priority for ts in new}
            ext.update_graph(s, client="client-0", keys=set(prio2), tasks=list(prio2), annotations={},
                             priority=prio2, dependencies={})
            assert ext.active, ext.reason
            s._transitions({ts.key: "waiting" for ts in sorted(new, key=lambda x: x.priority, reverse=True)}, {}, {},
                           "update-graph-2")
        ts = tss[t]
        s.stream_handlers["task-finished"](
            key=ts.key, worker=ts.processing_on.address, stimulus_id=f"tf-{t}", run_id=ts.run_id,
            nbytes=int(z["msg_nbytes"][i]), type=None, typename="int", metadata=None,
            startstops=[{"action": "compute", "start": float(z["msg_start"][i]), "stop": float(z["msg_stop"][i])}])
    ext._end_of_stimulus("end of stream")
    assert ext.active, ext.reason
    assert len(eng.graphs) == 1
    up = eng.graphs[0]
    assert np.array_equal(up["dep_ptr"], g2["dep_ptr"])
    for k in range(g2["n_tasks"]):  # earlier tasks by their engine index (-1 - index)
        row = g2["dep_idx"][g2["dep_ptr"][k]:g2["dep_ptr"][k + 1]].tolist()
        want = sorted(d if d >= 0 else -1 - ext.task_index[fkeys[-1 - d]] for d in row)
        assert up["dep_idx"][up["dep_ptr"][k]:up["dep_ptr"][k + 1]].tolist() == want, k
    host = 0
    if dep and not resync:  # the stimulus on the device: its inputs handed over first, no resync
        gst = [c for c in eng.calls if c[0] == "gstim"]
        assert len(gst) == 1 and not [c for c in eng.calls if c[0] == "sync"], eng.calls[-4:]
        assert ext.stats["graph_stimuli_on_device"] == 1 and ext.stats["resyncs"] == 0, ext.stats
        if "g2_lo_task" in z.files:  # a recompute: the extension's set orders are the generator's
            rp, li = z["g2_lo_rowptr"], z["g2_lo_idx"]
            want = sorted((int(t), int(k), tuple(li[rp[r]:rp[r + 1]].tolist()))
                          for r, (t, k) in enumerate(zip(z["g2_lo_task"].tolist(), z["g2_lo_kind"].tolist())))
            got = eng.graph_orders[-1]
            assert got is not None and sorted((t, k, tuple(q)) for t, k, q in got) == want
            assert ext.stats["graph_recomputes_on_device"] == 1, ext.stats
        if user_prio:  # every task's merged rank, before the stimulus
            ps = [c for c in eng.calls if c[0] == "prio"]
            assert len(ps) == 1 and eng.calls.index(ps[0]) < eng.calls.index(gst[0]), eng.calls[-3:]
            assert ps[0][1] == [int(z["g2_prio_all"][tidx[k]]) for k in ext.keys]
        if "restr_flags" in g2:  # the new tasks' valid workers, right before the stimulus
            rs = [c for c in eng.calls if c[0] == "restrict"]
            assert len(rs) == 1 and eng.calls.index(rs[0]) == eng.calls.index(gst[0]) - 1, eng.calls[-3:]
            _, rt, rrows, rfl = rs[0]
            rp, ri, rf = g2["restr_ptr"], g2["restr_idx"], g2["restr_flags"]
            want_r = sorted((ext.task_index[fkeys[N1 + k]], ri[rp[k]:rp[k + 1]].tolist(), int(rf[k]))
                            for k in np.flatnonzero(rf & 1))
            assert sorted(zip(rt, rrows, rfl)) == want_r
    if dep and resync:  # one resync, right after the submission: the fixture's dump
        syncs = [c for c in eng.calls if c[0] == "sync"]
        assert len(syncs) == 1 and (ext.stats["dependent_graphs"] + ext.stats["restricted_graphs"]
                                    + ext.stats["reranked_graphs"]) == 1, (len(syncs), ext.stats)
        if user_prio:  # every task's merged rank, handed over before the resync
            ps = [c for c in eng.calls if c[0] == "prio"]
            assert len(ps) == 1 and eng.calls.index(ps[0]) < eng.calls.index(syncs[0]), eng.calls[-3:]
            want_p = [int(z["g2_prio_all"][tidx[k]]) for k in ext.keys]
            assert ps[0][1] == want_p
        if "restr_flags" in g2:  # the new tasks' restrictions, handed over right after the resync
            rs = [c for c in eng.calls if c[0] == "restrict"]
            assert len(rs) == 1 and eng.calls.index(rs[0]) == eng.calls.index(syncs[0]) + 1, eng.calls[-3:]
            _, rt, rrows, rfl = rs[0]
            rp, ri, rf = g2["restr_ptr"], g2["restr_idx"], g2["restr_flags"]
            want_r = sorted((ext.task_index[fkeys[N1 + k]], ri[rp[k]:rp[k + 1]].tolist(), int(rf[k]))
                            for k in np.flatnonzero(rf & 1))
            assert sorted(zip(rt, rrows, rfl)) == want_r
        _, host, tasks, workers, glob = syncs[0]
        assert host == int(z["g2_nplaced"])
        ptr0 = {k: z[k + "_ptr"] for k in z.files if k.startswith("sync_") and k + "_ptr" in z.files}
        dump = {k: z[k][p[0]:p[1]] for k, p in ptr0.items()}
        row_of = {int(t): i for i, t in enumerate(dump["sync_tasks_task"].tolist())}
        fields = ("state", "remaining", "waiters", "processing_on", "nbytes", "long_running", "wanted")
        synced = set()
        for i, t in enumerate(tasks["task"].tolist()):
            f = tidx[ext.keys[t]]
            synced.add(f)
            assert all(tasks[fl][i] == dump["sync_tasks_" + fl][row_of[f]] for fl in fields), (t, f)
        for k in range(g2["n_tasks"]):  # every new task and every earlier task it depends on
            assert N1 + k in synced
            for d in g2["dep_idx"][g2["dep_ptr"][k]:g2["dep_ptr"][k + 1]]:
                assert (N1 + int(d) if d >= 0 else -1 - int(d)) in synced
        for part, rows in (("workers", workers), ("globals", glob)):
            for fl, v in rows.items():
                assert np.array_equal(np.atleast_1d(np.asarray(v)), dump[f"sync_{part}_{fl}"]), (part, fl)
    pnames = {i: nm for nm, i in ext.prefix_index.items()}
    gnames = {i: nm for nm, i in ext.group_index.items()}
    assert [pnames[i] for i in up["prefix_id"]] == [g2["prefix_names"][i] for i in g2["prefix_id"]]
    assert [gnames[i] for i in up["group_id"]] == [g2["group_names"][i] for i in g2["group_id"]]
    assert min(up["group_id"]) >= len(g["group_names"])  # new groups after the first graph's
    assert np.array_equal(up["prio"], np.arange(g2["n_tasks"]) + N1)
    n = len(exp["pl_task"])
    assert rec["task"] == exp["pl_task"].tolist()
    assert rec["worker"] == exp["pl_worker"].tolist()
    assert np.array_equal(np.array(rec["start"]).view(np.int64), exp["pl_start"].view(np.int64))
    assert ext.stats["device_decisions"] == n - host, (ext.stats, n, host)
    return dict(fixture=name, placements=n, graphs=ext.stats["graphs"], device_decisions=ext.stats["device_decisions"],
                host_placements=host, resyncs=ext.stats["resyncs"], active=ext.active, reason=ext.reason,
                graph_stimuli_on_device=ext.stats["graph_stimuli_on_device"])


def run_prefixes(name):
    """A ``svcpfx_*`` stream (gen_service.py prefixes): six later graphs, each with task
    prefixes of its own (75 over the stream), submitted through the plugins' update_graph
    hook. Where a graph would pass the engine's table (prefixes.PX) the extension compacts it
    (``_compact_prefixes``: dgp_remap_prefixes, then the dicts' resync) and stays active:
    every placement comes from the engine, validate=True re-derives each, and the remaps and
    resync rows equal the ones the generator recorded (the same prefixes.py on the reference
    state)."""
    import operator

    path = os.path.join(HERE, "golden", name)
    g, cfg, exp, meta = load_fixture(path)
    z = np.load(path, allow_pickle=False)
    g["keys"] = None
    sat = cfg["saturation"]
    sat = float("inf") if sat == "inf" else float(sat)
    dask.config.set({"distributed.scheduler.worker-saturation": sat})
    cfg = dict(cfg, saturation=sat)
    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    S = type(s)
    S.stimulus_task_finished = Scheduler.stimulus_task_finished
    S.handle_task_finished = Scheduler.handle_task_finished
    S.validate_key = lambda self, key, ts=None: None
    S.send_all = lambda self, client_msgs, worker_msgs: None
    fkeys = [ts.key for ts in tss]
    eng = EventEngine(exp, fkeys)
    ext = GPUPlacementExtension(s, engine_factory=lambda: eng, validate=True)
    eng.ext = ext
    s.stream_handlers = {}
    ext._install()
    priority = {ts.key: ts.priority for ts in tss}
    recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                     priority=priority, dependencies={})
    assert ext.active, ext.reason
    s._transitions(recs, {}, {}, "update-graph")
    cs = s.clients["client-0"]
    K = int(z["gk_n"])
    at = {int(z[f"g{k}_msg"]): k for k in range(K)}
    remaps_seen = 0
    for i, (t, w) in enumerate(zip(z["msg_task"].tolist(), z["msg_worker"].tolist())):
        if i in at:
            k = at[i]
            p = f"g{k}_"
            gk = dict(prefix_id=z[p + "prefix_local"], group_id=z[p + "group_local"],
                      prefix_names=z[p + "prefix_names"].tolist(), group_names=z[p + "group_names"].tolist(),
                      n_tasks=len(z[p + "prio"]))
            keys_k = G.make_keys(gk)
            base = len(tss)
            new = []
            for j, key in enumerate(keys_k):
                ts = s.new_task(key, (operator.add, (), {}), "released")
                tidx[key] = base + j
                ts.priority = (0, 2 + k, int(z[p + "prio"][j]))
                new.append(ts)
            dp, di = z[p + "dep_ptr"], z[p + "dep_idx"]
            for j, ts in enumerate(new):
                for d in di[dp[j]:dp[j + 1]]:
                    ts.add_dependency(new[int(d)])
                if z[p + "wanted"][j]:
                    ts.who_wants = {cs}
                    cs.wants_what.add(ts)
            eng.fkeys.extend(keys_k)
            tss.extend(new)
            n_calls = len(eng.calls)
            prio_k = {ts.key: ts.priority for ts in new}
            ext.update_graph(s, client="client-0", keys=set(prio_k), tasks=list(prio_k), annotations={},
                             priority=prio_k, dependencies={})
            assert ext.active, ext.reason
            rm = [c for c in eng.calls[n_calls:] if c[0] == "remap"]
            if p + "remap_slots" in z.files:  # the generator's remap and resync rows, the extension's too
                assert len(rm) == 1, eng.calls[n_calls:]
                remaps_seen += 1
                _, slots, defaults = rm[0]
                assert np.array_equal(slots, z[p + "remap_slots"]), k
                assert np.array_equal(np.asarray(defaults), z[p + "remap_defaults"]), k
                rows = [c for c in eng.calls[n_calls:] if c[0] == "sync_rows"]
                assert len(rows) == 1
                j0 = int(z[p + "remap_dump"])
                # group-indexed rows by group name (the fixture numbers groups in its graphs'
                # order, the extension in the order its ingestion meets them)
                fx_groups = list(meta["group_names"]) + [nm for kk in range(k) for nm in z[f"g{kk}_group_names"].tolist()]
                ext_groups = sorted(ext.group_index, key=ext.group_index.get)
                for part, got in (("workers", rows[0][1]), ("globals", rows[0][2])):
                    for fl, v in got.items():
                        pp = z[f"sync_{part}_{fl}_ptr"]
                        want = z[f"sync_{part}_{fl}"][pp[j0]:pp[j0 + 1]]
                        v = np.atleast_1d(np.asarray(v))
                        if fl.startswith("group_"):
                            eg = ext_groups[:len(v)]  # (the graph's own groups join after the resync)
                            assert len(eg) == len(fx_groups) == len(want), (k, fl)
                            v = dict(zip(eg, v.tolist()))
                            want = dict(zip(fx_groups, want.tolist()))
                            assert v == want, (k, part, fl)
                        else:
                            assert np.array_equal(v, want), (k, part, fl)
            else:
                assert not rm, (k, rm)
            s._transitions({ts.key: "waiting" for ts in sorted(new, key=lambda x: x.priority, reverse=True)}, {}, {},
                           f"update-graph-{k + 2}")
        ts = tss[t]
        s.stream_handlers["task-finished"](
            key=ts.key, worker=ts.processing_on.address, stimulus_id=f"tf-{t}", run_id=ts.run_id,
            nbytes=int(z["msg_nbytes"][i]), type=None, typename="int", metadata=None,
            startstops=[{"action": "compute", "start": float(z["msg_start"][i]), "stop": float(z["msg_stop"][i])}])
    ext._end_of_stimulus("end of stream")
    assert ext.active, ext.reason
    n = len(exp["pl_task"])
    assert rec["task"] == exp["pl_task"].tolist()
    assert rec["worker"] == exp["pl_worker"].tolist()
    assert np.array_equal(np.array(rec["start"]).view(np.int64), exp["pl_start"].view(np.int64))
    assert ext.stats["device_decisions"] == n, (ext.stats, n)
    return dict(fixture=name, placements=n, graphs=ext.stats["graphs"], device_decisions=ext.stats["device_decisions"],
                prefix_compactions=ext.stats["prefix_compactions"], remaps_checked=remaps_seen,
                prefixes_seen=len(ext.pnames), table=len(ext.prefix_index), resyncs=ext.stats["resyncs"],
                active=ext.active, reason=ext.reason)


class EventEngine(FixtureEngine):
    """FixtureEngine with the service-event calls: each consumes the fixture's placement
    count of its event and records what the extension passed."""

    def __init__(self, exp, fixture_keys):
        super().__init__(exp, fixture_keys)
        self.calls = []
        self.loss_orders = []  # the order rows of each lose_worker call
        self.loss_killed = []  # ... and its killed processing tasks
        self.graph_orders = []  # the order rows of each graph_stimulus call (None: plain)

    def _event(self, *call):
        assert self._posted is None, f"{call[0]} while a task-finished batch is posted"  # the engine refuses it
        self.calls.append(call)
        k = self.stim[self.k]
        self.n += k
        self.k += 1
        return k

    def add_replicas(self, t, w):
        for a, b in zip(t, w):
            self.who.setdefault(int(a), set()).add(int(b))
        return self._event("add", [int(x) for x in t], [int(x) for x in w])

    def remove_replicas(self, t, w):
        for a, b in zip(t, w):
            self.who.get(int(a), set()).discard(int(b))
        return self._event("remove", [int(x) for x in t], [int(x) for x in w])

    def set_worker_status(self, w, running):
        return self._event("status", int(w), int(running))

    def lose_worker(self, w, processing, held, order=(), killed=None):  # dgp_lose_worker_ordered
        for s_ in self.who.values():  # (the fixture's placements of that event)
            s_.discard(int(w))
        self.loss_orders.append([(int(t), int(k), [int(q) for q in seq]) for t, k, seq in order])
        self.loss_killed.append(sorted(int(t) for t, k in zip(processing, killed or ()) if k))
        return self._event("lose", int(w), [int(x) for x in processing], [int(x) for x in held])

    def long_running(self, t, cd):
        return self._event("long", int(t), float(cd))

    def reschedule(self, t):  # dgp_reschedule: the fixture's placements of that event
        return self._event("resched", int(t))

    def release_tasks(self, t, f):  # dgp_release_tasks: the fixture's placements of that event
        return self._event("release", [int(x) for x in t], [int(x) for x in f])

    def heartbeat(self, bw, ps, ds):
        return self._event("heartbeat", float(bw), [int(x) for x in ps], [float(x) for x in ds])

    def task_erred(self, t):
        return self._event("erred", int(t))

    # task inputs changed outside a transition (no placement of their own)
    def set_priorities(self, prio):
        self.calls.append(("prio", [int(x) for x in prio]))

    def set_rootish(self, t, v):
        self.calls.append(("rootish", [int(x) for x in t], [int(x) for x in v]))

    def update_restrictions(self, t, rows, flags):
        self.calls.append(("restrict", [int(x) for x in t], [[int(w) for w in r] for r in rows],
                           [int(x) for x in flags]))

    # state the engine follows without a placement of its own (no fixture event)
    def set_worker_flags(self, workers, idle, saturated):
        self.calls.append(("flags", [int(x) for x in workers], [int(x) for x in idle], [int(x) for x in saturated]))

    def set_wanted(self, task, wanted):
        self.calls.append(("wanted", [int(x) for x in task], [int(x) for x in wanted]))

    # resync after a stimulus the scheduler decided itself (one fixture event)
    def remove_worker(self, w):
        self.calls.append(("remove", int(w)))

    def remap_prefixes(self, task_prefix, prefix_default_duration):  # dgp_remap_prefixes: no placement
        self.calls.append(("remap", np.array(task_prefix, np.int32), [float(x) for x in prefix_default_duration]))

    def sync(self, placements, tasks, workers, globals_):
        if placements is None:  # the dicts in a compacted prefix numbering: no stimulus of its own
            assert tasks is None
            self.calls.append(("sync_rows", workers, globals_))
            return
        n = len(placements["task"])
        self.calls.append(("sync", n, tasks, workers, globals_))
        k = self.stim[self.k]
        assert n == k, (n, k)  # the scheduler's placements of that stimulus
        self.n += k
        self.k += 1
        # the replicas as the scheduler holds them after its stimulus (what the sync carries)
        e = self.ext
        for key, i in e.task_index.items():
            ts = e.scheduler.tasks.get(key)
            if ts is not None:
                self.who[i] = {e.worker_index[ws.address] for ws in ts.who_has or ()}
                self.nb[i] = ts.nbytes

    def sync_placements(self, *a):  # the extension calls sync(); these only mark the capability
        raise AssertionError("sync() expected")

    sync_tasks = sync_workers = sync_globals = sync_placements


class ResyncEventEngine(EventEngine):
    """The event engine without the worker-loss, reschedule and client-release operations:
    the extension hands those stimuli to the scheduler, then resynchronises the engine."""

    def __getattribute__(self, name):
        if name in ("lose_worker", "reschedule", "release_tasks"):
            raise AttributeError(name)
        return super().__getattribute__(name)


class GraphStimulusEngine(EventEngine):
    """EventEngine that runs a later graph's update_graph stimulus itself (dgp_graph_stimulus):
    the fixture's placement count of that event."""

    def graph_stimulus(self, order=None):
        self.graph_orders.append(order)
        return self._event("gstim")


def run_events(name, plain=False, resync_only=False):
    """A ``svcev_*`` stream (gen_service.py events): every event through the scheduler's own
    stream handler (add-keys, release-worker-data, worker-status-change, long-running,
    task-erred) or RPC handler (heartbeat_worker's placement part), wrapped by the
    extension, which must forward each to its engine call with the right arguments and stay
    active; every placement comes from the engine and validate=True re-derives it."""
    import math as _m

    from gen_service import (EV_ADD_KEYS, EV_ERRED, EV_FINISHED, EV_HEARTBEAT, EV_LONG_RUNNING, EV_PAUSE,
                             EV_RELEASE_DATA, EV_RELEASE_KEYS, EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RESTRICT,
                             EV_RESUME, EV_RETIRE, EV_RETIRE_REPLICA, EV_SHUFFLE_INIT, EV_LOSE_WORKER, EV_ERRED_RETRY,
                             EV_REFILL)

    from distributed_amd import sync as dsync

    path = os.path.join(HERE, "golden", name)
    g, cfg, exp, meta = load_fixture(path)
    z = np.load(path, allow_pickle=False)
    g["keys"] = None
    sat = cfg["saturation"]
    sat = float("inf") if sat == "inf" else float(sat)
    dask.config.set({"distributed.scheduler.worker-saturation": sat})
    cfg = dict(cfg, saturation=sat)
    s, tss, widx, rec, tidx = G.build_state(g, cfg)
    addr = {i: a for a, i in widx.items()}
    S = type(s)
    for nm in ("stimulus_task_finished", "handle_task_finished", "add_keys", "release_worker_data",
               "handle_worker_status_change", "handle_long_running", "handle_task_erred", "stimulus_task_erred"):
        setattr(S, nm, getattr(Scheduler, nm))
    S.validate_key = lambda self, key, ts=None: None
    S.send_all = lambda self, client_msgs, worker_msgs: None
    S.worker_send = lambda self, worker, msg: None
    s.extensions = {}
    resyncs = bool((z["ev_kind"] >= EV_REMOVE_WORKER).any())
    if resyncs:  # what Scheduler.remove_worker touches, as gen_service.replay_events sets it up
        import asyncio
        from collections import defaultdict
        from types import SimpleNamespace as NS

        from distributed.comm.addressing import get_address_host
        from distributed.core import Status

        S.remove_worker = Scheduler.remove_worker
        S.transition = Scheduler.transition  # a KilledWorker's processing -> erred (:5249-5256)
        S._reschedule = Scheduler._reschedule
        S.client_releases_keys = Scheduler.client_releases_keys
        S.stimulus_cancel = Scheduler.stimulus_cancel  # cancel-keys (:5364-5396)
        S.remove_client = Scheduler.remove_client  # close-client (:5727-5750)
        S.log_event = lambda self, topic, msg: None
        S.report = lambda self, msg, ts=None, client=None: None
        S.remove_resources = lambda self, address: None
        S.coerce_address = lambda self, a, resolve=True: a
        s.status = Status.running
        s.stream_comms = defaultdict(lambda: NS(send=lambda msg: None))
        s.rpc = NS(remove=lambda a: None)
        s.host_info = {}
        for a, ws in s.workers.items():
            hh = s.host_info.setdefault(get_address_host(a), {"addresses": set(), "nthreads": 0})
            hh["addresses"].add(a)
            hh["nthreads"] += ws.nthreads
        s.total_nthreads_history = []
        nm_ = os.path.basename(path)  # as gen_service.loss_allowed_failures
        s.allowed_failures = 0 if nm_.startswith("svcwl_killed0_") else 1 if nm_.startswith("svcwl_killed_") else 3
        s.bandwidth_workers = {}
        s.events = {}
        s._ongoing_background_tasks = NS(closed=False, call_later=lambda *a, **k: None)
        loop = asyncio.new_event_loop()

    def heartbeat_worker(*, address, metrics, executing=None, **kw):  # Scheduler.heartbeat_worker :4223-4252
        frac = 1 / len(s.workers)
        s.bandwidth = s.bandwidth * (1 - frac) + metrics["bandwidth"]["total"] * frac
        for key, duration in (executing or {}).items():
            if key in s.tasks:
                s.tasks[key].prefix.add_exec_time(duration)
        return {"status": "OK"}

    fkeys = [ts.key for ts in tss]
    eng = (FixtureEngine if plain else ResyncEventEngine if resync_only else EventEngine)(exp, fkeys)
    ext = GPUPlacementExtension(s, engine_factory=lambda: eng, validate=True)
    eng.ext = ext
    widx_all = dict(widx)
    tix = {k: i for i, k in enumerate(fkeys)}
    snap = {}

    def full_rows():
        return dsync.task_rows(s, fkeys, tix, widx_all)

    if not plain:  # every resync must carry each task whose state changed since the suspension
        orig_suspend = ext._suspend

        def suspend(reason):
            if not ext.suspended and "before" not in snap:
                snap["before"] = full_rows()
                snap["why"] = reason
            return orig_suspend(reason)

        ext._suspend = suspend
    s.stream_handlers = {"add-keys": s.add_keys, "release-worker-data": s.release_worker_data,
                         "worker-status-change": s.handle_worker_status_change,
                         "long-running": s.handle_long_running, "task-erred": s.handle_task_erred}
    if resyncs:
        s.stream_handlers["reschedule"] = s._reschedule
        s.stream_handlers["client-releases-keys"] = s.client_releases_keys
        s.stream_handlers["cancel-keys"] = s.stimulus_cancel
        s.stream_handlers["close-client"] = s.remove_client
    s.handlers = {"heartbeat_worker": heartbeat_worker}
    plugin = spec = None
    if (z["ev_kind"] == EV_SHUFFLE_INIT).any():  # the P2P shuffle plugin, bound to this state
        from types import SimpleNamespace as NS2

        from distributed.shuffle._core import barrier_key
        from distributed.shuffle._scheduler_plugin import ShuffleSchedulerPlugin

        S.set_restrictions = Scheduler.set_restrictions
        bar = next(ts for ts in tss if ts.prefix.name == "shuffle-barrier")

        class _View:  # what the plugin reads of its scheduler; set_restrictions goes to the (wrapped) method
            tasks = {barrier_key("fixture"): bar}

            def set_restrictions(self, worker):
                return s.set_restrictions(worker)

        plugin = ShuffleSchedulerPlugin.__new__(ShuffleSchedulerPlugin)
        plugin.scheduler = _View()
        spec = NS2(id="fixture")
        s.extensions["shuffle"] = plugin
    ext._install()
    priority = {ts.key: ts.priority for ts in tss}
    recs = {ts.key: "waiting" for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                     priority=priority, dependencies={})
    assert ext.active, ext.reason
    s._transitions(recs, {}, {}, "update-graph")
    want = []  # the engine calls the events imply
    n_sync = 0
    n_cancel = 0  # releases sent as cancel-keys (svccan_* leaves)
    n_retry = 0  # task-erred retries / stale runs (svcretry_*)
    on_device = set()  # EV_REMOVE_WORKER / EV_RESCHEDULE events the engine decided (dgp_lose_worker, dgp_reschedule)

    def check_sync():
        """The last engine call is the resync of this event: its worker / global rows equal
        the fixture's dump, and every task that changed since the suspension is a row."""
        nonlocal n_sync
        c = eng.calls[-1]
        assert c[0] == "sync", c[0]
        _, npl, tasks, workers, glob = c
        after = full_rows()
        before = snap.pop("before")
        snap["why_last"] = snap.pop("why", None)
        fields = ("state", "remaining", "waiters", "processing_on", "nbytes", "long_running", "wanted")
        hp_a, hi_a, hp_b, hi_b = after["holder_ptr"], after["holder_idx"], before["holder_ptr"], before["holder_idx"]
        changed = {i for i in range(len(fkeys))
                   if any(after[f][i] != before[f][i] for f in fields)
                   or list(hi_a[hp_a[i]:hp_a[i + 1]]) != list(hi_b[hp_b[i]:hp_b[i + 1]])}
        synced = set(tasks["task"].tolist())
        miss = sorted(changed - synced)
        assert not miss, [(t, {f: (before[f][t], after[f][t]) for f in fields}) for t in miss[:3]] + [snap.get("why_last")]
        for i, t in enumerate(tasks["task"].tolist()):  # the rows sent are the scheduler's state
            assert all(tasks[f][i] == after[f][t] for f in fields), t
        for part, rows in (("workers", workers), ("globals", glob)):
            for f, v in rows.items():
                key = f"sync_{part}_{f}"
                ptr = z[key + "_ptr"]
                assert np.array_equal(np.atleast_1d(np.asarray(v)), z[key][ptr[n_sync]:ptr[n_sync + 1]]), (part, f)
        n_sync += 1
    hp, ht, hd = z["hb_ptr"], z["hb_task"], z["hb_dur"]
    nbytes_bw = None
    for i, kd in enumerate(z["ev_kind"].tolist()):
        t, w, x = int(z["ev_task"][i]), int(z["ev_worker"][i]), float(z["ev_x"][i])
        sid = f"ev-{i}"
        H = s.stream_handlers
        if kd == EV_FINISHED:
            ts = tss[t]
            H["task-finished"](key=ts.key, worker=addr[w], stimulus_id=sid, run_id=ts.run_id,
                               nbytes=int(z["ev_nbytes"][i]), type=None, typename="int", metadata=None,
                               startstops=[{"action": "compute", "start": float(z["ev_start"][i]),
                                            "stop": float(z["ev_stop"][i])}])
        elif kd == EV_ADD_KEYS:
            H["add-keys"](worker=addr[w], keys=[tss[t].key], stimulus_id=sid)
            want.append(("add", [t], [w]))
        elif kd == EV_RELEASE_DATA:
            H["release-worker-data"](key=tss[t].key, worker=addr[w], stimulus_id=sid)
            want.append(("remove", [t], [w]))
        elif kd in (EV_PAUSE, EV_RESUME):
            H["worker-status-change"](status="running" if kd == EV_RESUME else "paused", worker=addr[w],
                                      stimulus_id=sid)
            want.append(("status", w, 1 if kd == EV_RESUME else 0))
        elif kd == EV_LONG_RUNNING:
            ts = tss[t]
            H["long-running"](key=ts.key, worker=addr[w], compute_duration=None if _m.isnan(x) else x,
                              stimulus_id=sid)
            want.append(("long", t, x))
        elif kd == EV_HEARTBEAT:
            ex = {tss[int(q)].key: float(d) for q, d in zip(ht[hp[i]:hp[i + 1]], hd[hp[i]:hp[i + 1]])}
            # the total that makes the reference's EWMA give the recorded bandwidth
            frac = 1 / len(s.workers)
            total = (x - s.bandwidth * (1 - frac)) / frac
            bw0 = s.bandwidth
            s.handlers["heartbeat_worker"](address=addr[w], metrics={"bandwidth": {"total": total}},
                                           executing=ex)
            assert s.bandwidth == x or abs(s.bandwidth - x) <= 1e-6 * x, (s.bandwidth, x)
            ps = [int(g["prefix_id"][int(q)]) for q in ht[hp[i]:hp[i + 1]]]
            if s.bandwidth != bw0 or ps:
                want.append(("heartbeat", float(s.bandwidth), ps, [float(d) for d in hd[hp[i]:hp[i + 1]]]))
            elif ext.active:
                eng.k += 1  # nothing changed: no engine call; the fixture's count for it is 0
        elif kd == EV_ERRED:
            ts = tss[t]
            H["task-erred"](key=ts.key, worker=addr[w], stimulus_id=sid, run_id=ts.run_id, exception=None,
                            traceback=None)
            want.append(("erred", t))
        elif kd == EV_ERRED_RETRY:  # a retry (ev_x 0) or a stale run (1): reschedule + refill on the engine
            ts = tss[t]
            stale = bool(x)
            if not stale:
                ts.retries = 1
            er0 = ext.stats["erred_retries"]
            H["task-erred"](key=ts.key, worker=addr[w], stimulus_id=sid, run_id=ts.run_id - 1 if stale else ts.run_id,
                            exception=None, traceback=None)
            assert ext.stats["erred_retries"] == er0 + 1 and not ext.suspended, (i, ext.stats, ext.suspend_reason)
            want.append(("resched", ext.task_index[fkeys[t]]))
            want.append(("release", [], []))
            n_retry += 1
        elif kd == EV_REFILL:  # consumed by the EV_ERRED_RETRY before it (the handler's refill)
            pass
        elif kd == EV_SHUFFLE_INIT:  # the first transfer runs: _ensure_output_tasks_are_non_rootish
            plugin._ensure_output_tasks_are_non_rootish(spec)
            ts_ = sorted(ext.task_index[fkeys[int(q)]] for q in ht[hp[i]:hp[i + 1]])
            want.append(("rootish", ts_, [0] * len(ts_)))
            eng.k += 1  # the fixture's count for it (no placement)
        elif kd == EV_RESTRICT:  # restrict_task -> _set_restriction -> Scheduler.set_restrictions
            plugin._set_restriction(tss[t], addr[w])
            want.append(("restrict", [ext.task_index[fkeys[t]]], [[w]], [1]))
            eng.k += 1
        elif kd == EV_RETIRE_REPLICA:  # made by the EV_RETIRE that follows (remove_worker's replica drops)
            want.append(("remove", [t], [w]))
        elif kd == EV_RETIRE:  # a drained worker leaves: no transition, followed on the device
            rs0 = ext.stats["resyncs"]
            loop.run_until_complete(s.remove_worker(addr[w], stimulus_id=sid))
            want.append(("remove", w))
            assert ext.stats["resyncs"] == rs0 and not ext.suspended, (i, ext.stats)
            eng.k += 1  # the fixture's count for it (no placement)
        elif kd == EV_LOSE_WORKER:  # a worker lost with work on it: the engine decides the stimulus
            rs0, lw0 = ext.stats["resyncs"], ext.stats["workers_lost_on_device"]
            lst = [int(q) for q in ht[hp[i]:hp[i + 1]]]
            loop.run_until_complete(s.remove_worker(addr[w], stimulus_id=sid))
            want.append(("lose", w, lst[:int(x)], lst[int(x):]))
            assert ext.stats["resyncs"] == rs0 and ext.stats["workers_lost_on_device"] == lw0 + 1, (i, ext.stats)
            assert not ext.suspended, (i, ext.suspend_reason)
            if "lo_evptr" in z.files:  # the extension's set orders are the generator's (same hash seed)
                ep, rp, li = z["lo_evptr"], z["lo_rowptr"], z["lo_idx"]
                rows = [(int(z["lo_task"][r]), int(z["lo_kind"][r]), li[rp[r]:rp[r + 1]].tolist())
                        for r in range(ep[i], ep[i + 1])]
                assert sorted(set((t, k, tuple(q)) for t, k, q in eng.loss_orders[-1])) == \
                    sorted(set((t, k, tuple(q)) for t, k, q in rows)), (i, eng.loss_orders[-1], rows)
                kp = z["lo_kptr"]
                assert eng.loss_killed[-1] == sorted(z["lo_ktask"][kp[i]:kp[i + 1]].tolist()), i
        elif kd in (EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS):
            if kd == EV_REMOVE_WORKER:
                lw0 = ext.stats["workers_lost_on_device"]
                loop.run_until_complete(s.remove_worker(addr[w], stimulus_id=sid))
                if ext.stats["workers_lost_on_device"] > lw0:  # a loss the engine restates: decided there
                    assert eng.calls[-1][:2] == ("lose", w), eng.calls[-1]
                    want.append(eng.calls[-1])
                    on_device.add(i)
                    n_sync += 1  # the fixture's resync rows of this event are not needed
                    snap.pop("before", None)
                    continue
                want.append(("remove", w))
            elif kd == EV_RESCHEDULE:
                rs0 = ext.stats["reschedule"]
                H["reschedule"](key=tss[t].key, worker=addr[w], stimulus_id=sid)
                if ext.stats["reschedule"] > rs0:  # decided by the engine (dgp_reschedule): no resync
                    assert eng.calls[-1] == ("resched", ext.task_index[fkeys[t]]), eng.calls[-1]
                    want.append(eng.calls[-1])
                    on_device.add(i)
                    n_sync += 1  # the fixture's resync rows of this event are not needed
                    snap.pop("before", None)
                    continue
            else:
                rl0 = ext.stats["release_tasks"]
                cs0 = s.clients["client-0"]
                if name.startswith("svccan_") and not tss[t].dependents and tss[t].who_wants == {cs0}:
                    # a wanted leaf: Client.cancel's cancel-keys, whose stimulus_cancel releases it
                    # through Scheduler.client_releases_keys (the extension's per-instance wrapper)
                    H["cancel-keys"](keys=[tss[t].key], client="client-0")
                    n_cancel += 1
                else:
                    H["client-releases-keys"](keys=[tss[t].key], client="client-0", stimulus_id=sid)
                if ext.stats["release_tasks"] > rl0:  # followed by the engine (dgp_release_tasks): no resync
                    c = eng.calls[-1]
                    assert c[0] == "release", c
                    if "rk_evptr" in z.files:  # the extension's closure is the generator's
                        rp = z["rk_evptr"]
                        want_t = [ext.task_index[fkeys[q]] for q in z["rk_task"][rp[i]:rp[i + 1]].tolist()]
                        # in the scheduler's transition order (dgp_release_tasks applies them in it)
                        assert list(zip(c[1], c[2])) == list(zip(want_t, z["rk_forget"][rp[i]:rp[i + 1]].tolist())), i
                    want.append(c)
                    on_device.add(i)
                    n_sync += 1
                    snap.pop("before", None)
                    continue
            if not plain:
                check_sync()
                want.append(eng.calls[-1])
        if plain:  # an engine without the event calls: the first event hands placement back
            if kd != EV_FINISHED:
                assert not ext.active and "not modelled" in ext.reason, (i, kd, ext.reason)
            continue
        assert ext.active, (i, kd, ext.reason)
    ext._end_of_stimulus("end of stream")
    n = len(exp["pl_task"])
    if plain:  # the scheduler's own decisions from the fallback on: still the reference's
        assert rec["task"] == exp["pl_task"].tolist() and rec["worker"] == exp["pl_worker"].tolist()
        assert 0 < ext.stats["device_decisions"] < n, ext.stats
        return dict(fixture=name, placements=n, device_decisions=ext.stats["device_decisions"], active=ext.active,
                    reason=ext.reason)
    assert ext.active, ext.reason
    got = [c for c in eng.calls]
    assert len(got) == len(want), (len(got), len(want))
    for a, b in zip(got, want):
        assert a[0] == b[0], (a, b)
        if a[0] == "long":
            assert a[1] == b[1] and (a[2] == b[2] or (_m.isnan(a[2]) and _m.isnan(b[2]))), (a, b)
        elif a[0] == "sync":
            assert a is b
        elif a[0] == "heartbeat":
            assert a[2] == b[2] and a[3] == b[3], (a, b)
        else:
            assert a == b, (a, b)
    assert rec["task"] == exp["pl_task"].tolist()
    assert rec["worker"] == exp["pl_worker"].tolist()
    assert np.array_equal(np.array(rec["start"]).view(np.int64), exp["pl_start"].view(np.int64))
    # the resync stimuli's placements are the scheduler's own, every other one the engine's
    host = sum(int(exp["stim_nplaced"][1 + i]) for i, kd in enumerate(z["ev_kind"].tolist())
               if kd in (EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS) and i not in on_device)
    assert ext.stats["device_decisions"] == n - host, (ext.stats, n, host)
    return dict(fixture=name, placements=n, events=len(want), device_decisions=ext.stats["device_decisions"],
                host_placements=host, resyncs=ext.stats["resyncs"], active=ext.active, reason=ext.reason,
                calls=dict(ext.stats), cancels=n_cancel, retries=n_retry)


class NullEngine:
    """The engine interface with nothing behind it: times the extension's own graph
    ingestion (TaskState -> the engine's arrays) apart from any engine."""

    def load(self, g, config, results=True):
        self.graph = g

    def set_resident(self, on=True):
        pass

    def set_task_messages(self, on=True):
        pass

    def update_graph(self):
        return 0

    def num_placements(self):
        return 0

    def close(self):
        pass


def run_ingest(n, workers=1024, repeat=3):
    """f4 ingestion: the extension's update_graph hook on an n-task C2-shaped graph of
    reference TaskStates (graph_from_tasks: ordering, dependency CSR, prefix / group /
    wanted / _rootish / restriction columns, and the extension's own index tables), with an
    engine that does nothing; the upload is checked against the graph it was built from."""
    from distributed_amd import graphs

    g = graphs.random_dag(n, workers, seed=5)
    g["keys"] = None
    s, tss, widx, rec, tidx = G.build_state(g, {"bandwidth": 100_000_000})
    fkeys = [ts.key for ts in tss]
    # as Scheduler.update_graph hands it to the plugins: descending priority (:4601-4611)
    priority = {ts.key: ts.priority for ts in sorted(tss, key=lambda t: t.priority, reverse=True)}
    best = None
    for _ in range(repeat):
        eng = NullEngine()
        ext = GPUPlacementExtension(s, engine_factory=lambda: eng)
        s.stream_handlers = {}
        ext._install()
        t0, c0 = _time.perf_counter(), _time.process_time()
        ext.update_graph(s, client="client-0", keys=set(priority), tasks=list(priority), annotations={},
                         priority=priority, dependencies={})
        dt, dc = _time.perf_counter() - t0, _time.process_time() - c0
        assert ext.active, ext.reason
        check_upload(eng.graph, ext.keys, g, fkeys)
        best = min(best or (dt, dc), (dt, dc))
    return dict(mode="ingest", n_tasks=n, n_workers=workers, n_edges=int(g["dep_ptr"][-1]),
                seconds=round(best[0], 4), us_per_task=round(1e6 * best[0] / n, 3),
                cpu_us_per_task=round(1e6 * best[1] / n, 3))


if __name__ == "__main__":
    import warnings

    warnings.filterwarnings("ignore")
    args = sys.argv[1:]
    diverge = "--diverge" in args
    plain = "--plain" in args
    stream = "--stream" in args
    for nm in [a for a in args if not a.startswith("--")]:
        if "--ingest" in args:
            print(json.dumps(run_ingest(int(nm))), flush=True)
            continue
        if "--ab" in args:
            print(json.dumps(run_ab(nm)), flush=True)
            continue
        fn = (run_joins if nm.startswith("svcaddw_") else (lambda x: run_second_graph(x, "--resync" in args))
              if nm.startswith(("svcgraph_", "svcgdep_", "svcgrst_", "svcgprio_", "svcgrec_"))
              else (lambda x: run_events(x, plain, "--resync-only" in args)) if nm.startswith(("svcev_", "svcrs_", "svcrt_", "svcwl_", "svcp2p_", "svcrel_", "svccan_", "svcretry_"))
              else run_prefixes if nm.startswith("svcpfx_")
              else None)
        print(json.dumps(fn(nm) if fn else run(nm, diverge, stream=stream,
                                               plain="plugin" if "--plugin" in args else plain,
                                               validate="--novalidate" not in args)), flush=True)
