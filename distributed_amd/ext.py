"""The drop-in Scheduler extension: dask.distributed's placement decisions from the MI355X
engine, behind the scheduler's own extension / plugin / transition-table API.

Register it like any scheduler extension (``distributed/scheduler.py:178-193``,
``:3890-3897``)::

    Scheduler(extensions={**DEFAULT_EXTENSIONS, "gpu-placement": GPUPlacementExtension})

or attach it to a running scheduler with ``GPUPlacementExtension(scheduler)``. Client
submission and workers are unchanged.

How it plugs in (the reference's interfaces, ``/root/reference/distributed/``):

* ``SchedulerPlugin`` hooks (``diagnostics/plugin.py:74-209``), registered with
  ``Scheduler.add_plugin`` (``scheduler.py:5940``) exactly like ``WorkStealing``
  (``stealing.py:108``): ``update_graph`` uploads the new runnable tasks (CSR dependencies,
  priorities, prefixes, groups, who_wants, ``_rootish``) and runs the engine's update_graph
  stimulus; ``add_worker`` / ``remove_worker`` / ``restart`` keep the engine's worker table.
* the instance ``_TRANSITIONS_TABLE`` (the class table ``scheduler.py:2889-2913`` is read
  through ``self`` at ``:1955``): ``("waiting", "processing")`` and ``("queued",
  "processing")`` take the worker the engine chose instead of calling
  ``decide_worker_rootish_queuing_enabled / _disabled`` / ``decide_worker_non_rootish``
  (``:2135-2311``); everything after the decision is the reference's own code
  (``_add_to_processing`` :3199, ``_task_to_msg`` :3421).
* ``stream_handlers["steal-response"]`` (``stealing.py:121``): the stealing extension's
  ``move_task_confirm`` (``:333-399``) runs as before; when it moved a processing task to
  the thief (the "confirm" branch ``:376-384``) the engine moves it too (``dgp_move_task``),
  so the device state follows confirmed steals.
* ``stream_handlers["task-finished"]`` (``:3769``): each message goes to the engine first
  (``dgp_tasks_finished``: stale / duplicate checks, completion, frontier release,
  frontier placement and queue refill on the device), then to the reference
  ``Scheduler.handle_task_finished`` (``:5783-5797``), whose transitions consume the
  engine's decisions in order.

The engine replays the scheduler's own stimulus sequence, so its placements come out in
the order the Python transitions ask for them. Every decision is checked against that
order: a task the engine did not place, or placed in another order, means the two have
diverged (a transition the engine does not model: worker loss, rescheduling, recompute,
restrictions). The extension then logs it, stops asking the engine and the scheduler
continues on its own Python decisions (``fallback``); ``validate=True`` also computes the
reference decision for every placement and raises on any difference (tests).
"""
from __future__ import annotations

import logging
import math
from collections import Counter, deque

import numpy as np

try:  # the plugin base class when dask.distributed is importable; plain object otherwise
    from distributed.diagnostics.plugin import SchedulerPlugin
except Exception:  # pragma: no cover - the GPU box has no dask
    SchedulerPlugin = object

logger = logging.getLogger("distributed_amd.ext")

_REF = object()  # "no engine decision: run the reference's own transition"


def _compute_interval(startstops):
    """The "compute" startstop of a task-finished message (TaskGroup.add_duration is fed
    every startstop; only "compute" moves TaskPrefix.duration_average, :977-985)."""
    for ss in startstops or ():
        if ss.get("action") == "compute":
            return float(ss["start"]), float(ss["stop"])
    return math.nan, math.nan


def graph_from_tasks(tss, nthreads, valid_workers=None, worker_index=None):
    """TaskState objects -> the engine's graph arrays (the layout of distributed_amd/graphs.py).

    Tasks are indexed in ascending ``TaskState.priority`` (so ``prio`` is their rank: unique
    and topological for dask.order priorities); dependencies must be among ``tss``.
    Prefixes / groups get ids in first-seen order; ``prefix_default_dur`` is each
    ``TaskPrefix.duration_average`` now (default-task-durations or -1).

    Restrictions: with ``valid_workers`` (``SchedulerState.valid_workers``, scheduler.py
    :3043-3107, which resolves worker / host / resource restrictions) and ``worker_index``
    (address -> engine worker index), every task with restrictions gets its valid set as
    ascending indices (``restr_ptr`` / ``restr_idx``) and ``restr_flags`` (1: restricted,
    2: loose_restrictions)."""
    tss = sorted(tss, key=lambda ts: ts.priority)
    index = {ts.key: i for i, ts in enumerate(tss)}
    n = len(tss)
    rows = []
    for ts in tss:
        try:
            rows.append(sorted(index[d.key] for d in ts.dependencies))
        except KeyError as e:
            raise ValueError(f"dependency {e} of {ts.key!r} is not in the uploaded graph") from None
    pnames, gnames, gpref = {}, {}, []
    pid = np.zeros(n, np.int32)
    gid = np.zeros(n, np.int32)
    pdur = []
    for i, ts in enumerate(tss):
        p = ts.prefix.name
        if p not in pnames:
            pnames[p] = len(pnames)
            pdur.append(float(ts.prefix.duration_average))
        g = ts.group.name
        if g not in gnames:
            gnames[g] = len(gnames)
            gpref.append(pnames[p])
        pid[i] = pnames[p]
        gid[i] = gnames[g]
    ptr = np.zeros(n + 1, np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    g = dict(
        n_tasks=n,
        dep_ptr=ptr,
        dep_idx=np.array([d for r in rows for d in r], np.int32),
        prio=np.arange(n, dtype=np.int64),
        prefix_id=pid,
        group_id=gid,
        prefix_names=list(pnames),
        group_names=list(gnames),
        group_prefix=np.array(gpref, np.int32),
        prefix_default_dur=np.array(pdur, np.float64),
        wanted=np.array([1 if ts.who_wants else 0 for ts in tss], np.uint8),
        rootish_override=np.array([-1 if ts._rootish is None else int(bool(ts._rootish)) for ts in tss], np.int8),
        nthreads=np.asarray(nthreads, np.int32),
        # completion reports arrive with the task-finished messages (service mode)
        nbytes=np.full(n, -1, np.int64),
        start=np.zeros(n),
        stop=np.zeros(n),
    )
    if valid_workers is not None:
        flags = np.zeros(n, np.uint8)
        vrows = [[] for _ in range(n)]
        for i, ts in enumerate(tss):
            if ts.worker_restrictions or ts.host_restrictions or ts.resource_restrictions:
                vw = valid_workers(ts)
                if vw is None:  # restrictions that exclude nobody
                    continue
                flags[i] = 1 | (2 if ts.loose_restrictions else 0)
                vrows[i] = sorted(worker_index[ws.address] for ws in vw)
        if flags.any():
            rp = np.zeros(n + 1, np.int64)
            rp[1:] = np.cumsum([len(r) for r in vrows])
            g.update(restr_ptr=rp, restr_idx=np.array([w for r in vrows for w in r], np.int32), restr_flags=flags)
    return g, [ts.key for ts in tss]


class GPUPlacementExtension(SchedulerPlugin):
    """Scheduler extension that takes placement decisions from the HIP engine."""

    name = "gpu-placement"

    def __init__(self, scheduler, *, device: int = 0, engine_factory=None, validate: bool = False):
        self.scheduler = scheduler
        self.device = device
        self.engine_factory = engine_factory
        self.validate = validate
        self.engine = None
        self.active = True
        self.reason = None        # why the extension fell back to the reference decisions
        self.keys: list = []      # engine task index -> key
        self.task_index: dict = {}
        self.workers: list = []   # engine worker index -> address
        self.worker_index: dict = {}
        self.dev_run: dict = {}   # key -> placement-log position of its current placement
        self.pending: deque = deque()  # (task index, worker index) in placement order
        self.n_fetched = 0
        self.stats = Counter()
        if hasattr(scheduler, "add_plugin"):
            scheduler.add_plugin(self, name=self.name)
        self._install()

    # ---------------------------------------------------------------- plumbing
    def _install(self):
        s = self.scheduler
        table = dict(type(s)._TRANSITIONS_TABLE)
        ref_wp = table[("waiting", "processing")]
        ref_qp = table[("queued", "processing")]

        def waiting_processing(sched, key, stimulus_id, **kwargs):
            return self._transition_waiting_processing(sched, key, stimulus_id, ref_wp)

        def queued_processing(sched, key, stimulus_id, **kwargs):
            return self._transition_queued_processing(sched, key, stimulus_id, ref_qp)

        table[("waiting", "processing")] = waiting_processing
        table[("queued", "processing")] = queued_processing
        s._TRANSITIONS_TABLE = table  # per instance: the class table stays untouched
        handlers = getattr(s, "stream_handlers", None)
        if handlers is not None:
            handlers["task-finished"] = self.handle_task_finished
        self._wrap_stealing()

    def _wrap_stealing(self):
        """Follow confirmed steals: wrap the stealing extension's ``move_task_confirm``
        (stealing.py:333-399), which is also its ``steal-response`` stream handler (:121)."""
        s = self.scheduler
        st = (getattr(s, "extensions", None) or {}).get("stealing")
        if st is None or getattr(st, "_gpu_placement_wrapped", False):
            return
        orig = st.move_task_confirm

        async def move_task_confirm(*, key, state, stimulus_id, worker=None):
            ts = s.tasks.get(key)
            before = ts.processing_on if ts is not None and ts.state == "processing" else None
            try:
                await orig(key=key, state=state, stimulus_id=stimulus_id, worker=worker)
            finally:
                ts = s.tasks.get(key)
                if before is not None and ts is not None:
                    if ts.state == "processing" and ts.processing_on is not None and ts.processing_on is not before:
                        self.task_moved(ts, ts.processing_on)
                    elif ts.state != "processing":  # "reschedule" (:365-376): not modelled on the device
                        self.fallback(f"steal of {key!r} rescheduled it")

        st.move_task_confirm = move_task_confirm
        if getattr(s, "stream_handlers", None) is not None and "steal-response" in s.stream_handlers:
            s.stream_handlers["steal-response"] = move_task_confirm
        st._gpu_placement_wrapped = True

    def task_moved(self, ts, thief):
        """A confirmed steal moved processing ``ts`` to ``thief`` (a WorkerState)."""
        if not self.active or self.engine is None:
            return
        t = self.task_index.get(ts.key)
        w = self.worker_index.get(thief.address)
        if t is None or w is None:
            self.fallback(f"steal of {ts.key!r} to {thief.address}: not in the engine's tables")
            return
        try:
            self.engine.move_task(t, w)
            self.stats["steals_confirmed"] += 1
        except Exception as e:
            self.fallback(f"move_task: {e}")

    def fallback(self, reason: str):
        """Stop asking the engine; the scheduler continues on its own decisions."""
        if self.active:
            logger.warning("gpu-placement: falling back to the scheduler's own placement: %s", reason)
        self.active = False
        self.reason = reason
        self.pending.clear()

    def _config(self):
        from distributed import scheduler as sched_mod

        s = self.scheduler
        sat = s.WORKER_SATURATION
        return {"bandwidth": int(s.bandwidth), "default_data_size": int(sched_mod.DEFAULT_DATA_SIZE),
                "unknown_duration": float(s.UNKNOWN_TASK_DURATION),
                "saturation": "inf" if math.isinf(sat) else float(sat)}

    def _fetch(self):
        """Queue the engine's new placements (the decisions the transitions will ask for)."""
        n = self.engine.num_placements()
        if n > self.n_fetched:
            pl = self.engine.placements(self.n_fetched, n - self.n_fetched)
            for j, (t, w) in enumerate(zip(pl["pl_task"].tolist(), pl["pl_worker"].tolist())):
                self.pending.append((t, w))
                self.dev_run[self.keys[t]] = self.n_fetched + j
            self.n_fetched = n

    def _end_of_stimulus(self, what: str):
        if self.active and self.pending:
            t, w = self.pending[0]
            self.fallback(f"{what}: the engine placed {self.keys[t]!r} on {self.workers[w]} but the scheduler "
                          "did not ask for it")

    # ------------------------------------------------------- placement decisions
    def _decision(self, sched, ts, queued: bool):
        """The engine's worker for ``ts`` (a WorkerState), None (the engine did not place
        it in this stimulus: it stays / goes queued), or _REF (run the reference)."""
        if not self.active or self.engine is None:
            return _REF
        t = self.task_index.get(ts.key)
        if t is None:
            self.fallback(f"{ts.key!r} is not in the engine's graph")
            return _REF
        if self.pending and self.pending[0][0] == t:
            _, w = self.pending.popleft()
            self.stats["device_decisions"] += 1
            return sched.workers[self.workers[w]]
        if any(p[0] == t for p in self.pending):
            self.fallback(f"placement order differs at {ts.key!r}")
            return _REF
        # not placed by the engine: only a root-ish task under queuing may stay / go queued
        # (decide_worker_rootish_queuing_enabled found no slot, :2230-2245); anything else
        # is a transition the engine did not run
        if queued or (not math.isinf(sched.WORKER_SATURATION) and sched.is_rootish(ts)):
            self.stats["device_queued"] += 1
            return None
        # restrictions that no worker satisfies, not loose: the engine left it in
        # no-worker (decide_worker :8584-8586 -> _transition_waiting_no_worker :2761-2782)
        if ((ts.worker_restrictions or ts.host_restrictions or ts.resource_restrictions)
                and not ts.loose_restrictions and sched.valid_workers(ts) == set()):
            self.stats["device_no_worker"] += 1
            return None
        self.fallback(f"the engine did not place {ts.key!r}")
        return _REF

    def _reference_decision(self, sched, ts, queued: bool):
        if queued:
            return sched.decide_worker_rootish_queuing_enabled()
        if sched.is_rootish(ts):
            if math.isinf(sched.WORKER_SATURATION):
                return sched.decide_worker_rootish_queuing_disabled(ts)
            return sched.decide_worker_rootish_queuing_enabled()
        return sched.decide_worker_non_rootish(ts)

    def _check(self, sched, ts, ws, queued):
        if self.validate:
            ref = self._reference_decision(sched, ts, queued)
            if ref is not ws:
                raise AssertionError(f"gpu-placement: engine chose {ws and ws.address} for {ts.key!r}, "
                                     f"the reference {ref and ref.address}")

    def _transition_waiting_processing(self, sched, key, stimulus_id, ref):
        """_transition_waiting_processing (scheduler.py:2313-2336) with the engine's decision."""
        ts = sched.tasks[key]
        ws = self._decision(sched, ts, False)
        if ws is _REF:
            return ref(sched, key, stimulus_id)
        self._check(sched, ts, ws, False)
        if ws is None:
            if sched.is_rootish(ts) and not math.isinf(sched.WORKER_SATURATION):
                return {ts.key: "queued"}, {}, {}
            return {ts.key: "no-worker"}, {}, {}
        return sched._add_to_processing(ts, ws, stimulus_id=stimulus_id)

    def _transition_queued_processing(self, sched, key, stimulus_id, ref):
        """_transition_queued_processing (scheduler.py:2797-2808) with the engine's decision."""
        ts = sched.tasks[key]
        ws = self._decision(sched, ts, True)
        if ws is _REF:
            return ref(sched, key, stimulus_id)
        self._check(sched, ts, ws, True)
        if ws is None:
            return {}, {}, {}
        sched.queued.discard(ts)
        return sched._add_to_processing(ts, ws, stimulus_id=stimulus_id)

    # ----------------------------------------------------------- plugin hooks
    def update_graph(self, scheduler, *, client=None, keys=(), tasks=(), annotations=None, priority=None,
                     dependencies=None, **kwargs):
        """SchedulerPlugin.update_graph (diagnostics/plugin.py:74-109): runs before the
        scheduler transitions the new tasks (scheduler.py:4641-4653)."""
        if not self.active:
            return
        s = self.scheduler
        new = [s.tasks[k] for k in (priority or {}) if k in s.tasks and k not in self.task_index]
        if not new:
            return
        try:
            if self.engine is not None:
                self._add_graph(new)
                return
            self.workers = list(s.workers)
            self.worker_index = {a: i for i, a in enumerate(self.workers)}
            g, keys_ = graph_from_tasks(new, [s.workers[a].nthreads for a in self.workers], s.valid_workers,
                                        self.worker_index)
            self.keys = keys_
            self.task_index = {k: i for i, k in enumerate(keys_)}
            self.prefix_index = {nm: i for i, nm in enumerate(g["prefix_names"])}
            self.group_index = {nm: i for i, nm in enumerate(g["group_names"])}
            self.prefix_dur = list(g["prefix_default_dur"])
            self.group_prefix = list(g["group_prefix"])
            self.max_priority = max(ts.priority for ts in new)
            if self.engine_factory is not None:
                self.engine = self.engine_factory()
            else:
                from .engine import PlacementEngine

                self.engine = PlacementEngine(self.device)
            self.engine.load(g, self._config(), results=False)
            self.engine.update_graph()
            self._fetch()
            self.stats["graphs"] += 1
        except Exception as e:  # plugin errors are logged, not raised (scheduler.py:4652-4653)
            self.fallback(f"update_graph: {e}")

    def _add_graph(self, new):
        """A later update_graph (scheduler.py:4662-4751) on the running engine: the new
        tasks must not depend on earlier ones (graph_from_tasks raises otherwise) and must
        all follow them in priority (a new generation, :4713, with no user priority above
        the earlier graphs'); prefixes and groups map into the engine-wide tables."""
        s = self.scheduler
        g, keys_ = graph_from_tasks(new, [s.workers[a].nthreads for a in self.workers], s.valid_workers,
                                    self.worker_index)
        if "restr_flags" in g:
            raise NotImplementedError("worker restrictions in a later graph")
        if min(ts.priority for ts in new) <= self.max_priority:
            raise NotImplementedError("a later graph whose tasks do not all follow the earlier ones in priority")
        pmap = np.zeros(len(g["prefix_names"]), np.int32)
        for i, nm in enumerate(g["prefix_names"]):
            if nm not in self.prefix_index:
                self.prefix_index[nm] = len(self.prefix_index)
                self.prefix_dur.append(float(g["prefix_default_dur"][i]))
            pmap[i] = self.prefix_index[nm]
        gmap = np.zeros(len(g["group_names"]), np.int32)
        for i, nm in enumerate(g["group_names"]):
            if nm not in self.group_index:
                self.group_index[nm] = len(self.group_index)
                self.group_prefix.append(int(pmap[g["group_prefix"][i]]))
            gmap[i] = self.group_index[nm]
        n0 = len(self.keys)
        g2 = dict(dep_ptr=g["dep_ptr"], dep_idx=g["dep_idx"], prio=g["prio"] + n0, prefix_id=pmap[g["prefix_id"]],
                  group_id=gmap[g["group_id"]], wanted=g["wanted"], rootish_override=g["rootish_override"],
                  prefix_default_dur=np.array(self.prefix_dur, np.float64),
                  group_prefix=np.array(self.group_prefix, np.int32))
        self._end_of_stimulus("the previous stimulus")
        if not self.active:
            return
        self.engine.add_graph(g2)
        self.keys = self.keys + keys_
        self.task_index.update({k: n0 + i for i, k in enumerate(keys_)})
        self.max_priority = max(ts.priority for ts in new)
        self._fetch()
        self.stats["graphs"] += 1

    def add_worker(self, scheduler=None, worker=None):
        """SchedulerPlugin.add_worker (diagnostics/plugin.py): Scheduler.add_worker calls it
        after check_idle_saturated(ws) and before bulk_schedule_unrunnable_after_adding_worker /
        stimulus_queue_slots_maybe_opened (scheduler.py:4398-4420). The engine adds the worker
        and makes the queue refill; the scheduler's own refill then consumes those decisions.
        The engine's worker index order must stay the scheduler's (SortedDict address) order,
        so only a worker whose address sorts after every known one joins on the device."""
        if not self.active or self.engine is None or worker in self.worker_index:
            return
        if self.workers and worker < max(self.workers):
            self.fallback(f"add_worker({worker}): its address sorts before a known worker's")
            return
        s = self.scheduler
        try:
            self._end_of_stimulus("the previous stimulus")
            if not self.active:
                return
            self.engine.add_worker(int(s.workers[worker].nthreads))
            self.worker_index[worker] = len(self.workers)
            self.workers.append(worker)
            self._fetch()
            self.stats["workers_added"] += 1
        except Exception as e:
            self.fallback(f"add_worker({worker}): {e}")

    def remove_worker(self, scheduler=None, worker=None, **kwargs):
        if self.engine is not None and worker in self.worker_index:
            self.fallback(f"remove_worker({worker})")

    def restart(self, scheduler=None):
        self.close_engine()
        self.active = True
        self.reason = None

    def close_engine(self):
        if self.engine is not None and hasattr(self.engine, "close"):
            self.engine.close()
        self.engine = None
        self.keys, self.task_index, self.dev_run = [], {}, {}
        self.pending.clear()
        self.n_fetched = 0

    async def close(self):
        self.close_engine()

    # ------------------------------------------------------- task-finished
    def _message_fields(self, key, worker, msg):
        s = self.scheduler
        t = self.task_index.get(key, len(self.keys))  # unknown key: out of range = forgotten
        w = self.worker_index.get(worker, len(self.workers))
        ts = s.tasks.get(key)
        run = -2
        if ts is not None and key in self.dev_run and msg.get("run_id") == ts.run_id:
            run = self.dev_run[key]
        nbytes = msg.get("nbytes")
        a, b = _compute_interval(msg.get("startstops"))
        return t, w, run, -1 if nbytes is None else int(nbytes), a, b

    def handle_task_finished(self, key=None, worker=None, stimulus_id=None, **msg):
        """Stream handler "task-finished" (scheduler.py:3769 -> :5783-5797)."""
        self.handle_task_finished_batch([dict(msg, key=key, worker=worker, stimulus_id=stimulus_id)])

    def handle_task_finished_batch(self, msgs):
        """Several task-finished messages in arrival order: ONE engine call (one PCIe copy),
        then the reference handler for each, consuming the engine's decisions in order."""
        s = self.scheduler
        handler = type(s).handle_task_finished
        self._end_of_stimulus("the previous stimulus")
        if self.active and self.engine is not None and msgs:
            fields = [self._message_fields(m["key"], m["worker"], m) for m in msgs]
            cols = list(zip(*fields))
            try:
                status, _ = self.engine.tasks_finished(*cols)
                self._fetch()
                self.stats["messages"] += len(msgs)
                status = np.asarray(status)
                # DGP_TF_RELEASE / _IMPOSSIBLE / _UNSUPPORTED: the reference reschedules or
                # raises; the engine does not follow those transitions
                if np.any(status >= 3) and np.any((status != 4) & (status >= 3)):
                    self.fallback(f"task-finished answers {sorted(set(status.tolist()))} the engine does not run")
            except Exception as e:
                self.fallback(f"tasks_finished: {e}")
        for m in msgs:
            m = dict(m)
            handler(s, m.pop("key"), m.pop("worker"), m.pop("stimulus_id"), **m)
        self._end_of_stimulus("task-finished")
