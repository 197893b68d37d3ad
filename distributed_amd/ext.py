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
  stimulus; ``add_worker`` / ``remove_worker`` / ``restart`` keep the engine's worker table;
  ``transition`` is the catch-all described below.
* the instance ``_TRANSITIONS_TABLE`` (the class table ``scheduler.py:2889-2913`` is read
  through ``self`` at ``:1955``): ``("waiting", "processing")`` and ``("queued",
  "processing")`` take the worker the engine chose instead of calling
  ``decide_worker_rootish_queuing_enabled / _disabled`` / ``decide_worker_non_rootish``
  (``:2135-2311``); everything after the decision is the reference's own code
  (``_add_to_processing`` :3199, ``_task_to_msg`` :3421).
* ``stream_handlers["task-finished"]`` (``:3769``): each batch of messages goes to the
  engine first (``dgp_tasks_finished``: stale / duplicate checks, completion, frontier
  release, frontier placement and queue refill on the device), then to the reference
  ``Scheduler.handle_task_finished`` (``:5783-5797``), whose transitions consume the
  engine's decisions in order.
* every other stimulus that changes a placement input (``scheduler.py:3768-3792`` worker
  and client stream handlers, the ``heartbeat_worker`` RPC ``:4197-4252``,
  ``set_restrictions`` ``:7702``, ``SchedulerState.add_replica`` / ``remove_replica``
  ``:3148-3159`` from any caller, the stealing extension's ``balance`` and
  ``move_task_confirm`` ``stealing.py:333-503``) is followed on the device when the engine
  models it (``_ENGINE_EVENTS``) and otherwise ends GPU placement for the session, loudly.

Nothing diverges silently. The engine replays the scheduler's own stimulus sequence, so its
placements come out in the order the Python transitions ask for them, and every decision is
checked against that order; a transition the engine does not model (worker loss, erred
tasks, rescheduling, recompute, client releases, ...) is caught by the plugin
``transition`` hook; a queued task the engine left queued while the scheduler has an open
slot is a divergence too. The extension then logs it (``fallback``), stops asking the
engine and the scheduler continues on its own Python decisions. ``validate=True`` also
computes the reference decision for every placement and raises on any difference (tests).
"""
from __future__ import annotations

import asyncio
import bisect
import functools
import inspect
import logging
import math
from collections import Counter, deque
from itertools import chain, islice, repeat
from operator import attrgetter, lt, truth

import numpy as np

from . import loss, prefixes, sync

try:  # the plugin base class when dask.distributed is importable; plain object otherwise
    from distributed.diagnostics.plugin import SchedulerPlugin
except Exception:  # pragma: no cover - the GPU box has no dask
    SchedulerPlugin = object

logger = logging.getLogger("distributed_amd.ext")

_REF = object()  # "no engine decision: run the reference's own transition"

# transitions the engine runs itself inside a stimulus it follows (task-finished:
# processing -> memory, the releases of dependencies, the frontier and the queue refill;
# update_graph: released -> waiting -> processing / queued / no-worker)
_STIMULUS_TRANSITIONS = frozenset({
    ("processing", "memory"), ("memory", "released"), ("released", "waiting"), ("waiting", "processing"),
    ("waiting", "queued"), ("waiting", "no-worker"), ("queued", "processing")})
_UPDATE_GRAPH_TRANSITIONS = frozenset({
    ("released", "waiting"), ("waiting", "processing"), ("waiting", "queued"), ("waiting", "no-worker")})
_ADD_WORKER_TRANSITIONS = frozenset({("queued", "processing")})
# a removed worker keeps its engine index under this suffix: it sorts right after its address
# (no address has a NUL), so the list stays in address order if the address joins again
_REMOVED = "\x00removed"
# stimulus_queue_slots_maybe_opened after long-running / a worker running again (:4983-5023)
_REFILL_TRANSITIONS = _ADD_WORKER_TRANSITIONS
# task-erred (:5094-5127, :2630-2720): the task erred, its waiting dependents released then
# erred (the _transition fallback through "released", :1960-1980), dependencies nobody
# waits for released, then the queue refill
_ERRED_TRANSITIONS = frozenset({("processing", "erred"), ("waiting", "released"), ("released", "erred"),
                                ("memory", "released"), ("queued", "processing")})
# client-releases-keys (:5417-5430): memory -> released / forgotten, released -> forgotten,
# cancelled work -> released (dgp_release_tasks), then the queue refill
_RELEASE_TRANSITIONS = frozenset({("memory", "released"), ("memory", "forgotten"), ("released", "forgotten"),
                                  ("processing", "released"), ("waiting", "released"), ("queued", "released"),
                                  ("no-worker", "released"), ("queued", "processing")})
# reschedule (Scheduler._reschedule :7900-7924): processing -> released -> waiting, then
# decide_worker (dgp_reschedule)
_RESCHEDULE_TRANSITIONS = frozenset({("processing", "released"), ("released", "waiting"), ("waiting", "processing"),
                                     ("waiting", "queued"), ("waiting", "no-worker")})
# a worker lost with processing tasks / sole replicas (Scheduler.remove_worker :5233-5303):
# processing -> released (-> waiting through released, :1961-1984), memory -> released for the
# lost results and the recompute chains' released dependencies, released -> waiting, then
# decide_worker; a no-worker waiter through released; a KilledWorker's erred cascade
_LOSS_TRANSITIONS = frozenset({("processing", "released"), ("released", "waiting"), ("memory", "released"),
                               ("waiting", "processing"), ("waiting", "queued"), ("waiting", "no-worker"),
                               ("no-worker", "released")}) | _ERRED_TRANSITIONS - {("queued", "processing")}

# the placement inputs a stimulus other than task-finished / update_graph / add_worker can
# change, and the engine method that follows each on the device (PlacementEngine); an engine
# without the method (or one that raises) hands placement back to the scheduler
_ENGINE_EVENTS = ("add_replicas", "remove_replicas", "set_worker_status", "long_running", "heartbeat",
                  "set_worker_flags", "set_wanted", "task_erred", "update_restrictions", "set_rootish")


_SM = None


def _sched_mod():
    """distributed.scheduler, imported once (the compute-task message's TaskState run_id
    counter, time and ToPickle)."""
    global _SM
    if _SM is None:
        from distributed import scheduler

        _SM = scheduler
    return _SM


def _compute_interval(startstops):
    """The "compute" startstop of a task-finished message (TaskGroup.add_duration is fed
    every startstop; only "compute" moves TaskPrefix.duration_average, :977-985)."""
    for ss in startstops or ():
        if ss.get("action") == "compute":
            return float(ss["start"]), float(ss["stop"])
    return math.nan, math.nan


_PRIO, _KEY, _DEPS = attrgetter("priority"), attrgetter("key"), attrgetter("dependencies")
_GROUP, _PREFIX, _WANTS, _ROOTISH = attrgetter("group"), attrgetter("prefix"), attrgetter("who_wants"), attrgetter("_rootish")
_RESTR = (attrgetter("worker_restrictions"), attrgetter("host_restrictions"), attrgetter("resource_restrictions"))
_ROOTISH_CODE = {None: -1, False: 0, True: 1}


_FORCE_PY_INGEST = False  # tests: the Python passes even where the C library is built
_INGEST = []  # [ctypes function or None]: libdgpingest.so's dgp_ingest_columns, loaded once


def _ingest_lib():
    """dgp_ingest_columns (csrc/dgp_ingest.c, built by distributed_amd/build.py) through
    ctypes.PyDLL (the GIL stays held, its Python errors propagate); None when the library
    is not built (graph_from_tasks then runs its Python passes)."""
    if not _INGEST:
        import ctypes
        import os

        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdgpingest.so")
        fn = None
        if os.path.exists(path):
            fn = ctypes.PyDLL(path).dgp_ingest_columns
            P = ctypes.c_void_p
            fn.argtypes = [ctypes.py_object, ctypes.py_object, P, P, ctypes.c_int64, P, P, P, P, P, P, P, P]
            fn.restype = ctypes.c_int64
        _INGEST.append(fn)
    return _INGEST[0]


def _columns_c(fn, tss):
    """The per-task columns in one C pass (dgp_ingest_columns): (dependency counts, flat
    dependency ids in set order (-1 - m: misses[m], outside ``tss``), misses, prefix ids,
    first task per prefix, group ids, first task per group, wanted, rootish code,
    restriction bits)."""
    n = len(tss)
    cnt = np.empty(n, np.int64)
    pid, gid = np.empty(n, np.int32), np.empty(n, np.int32)
    pfirst, gfirst = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32)
    nid = np.zeros(2, np.int32)
    wanted, rootish, restr = np.empty(n, np.uint8), np.empty(n, np.int8), np.empty(n, np.uint8)
    cap = 4 * n + 16
    while True:
        misses = []
        dflat = np.empty(cap, np.int64)
        e = fn(tss, misses, cnt.ctypes.data, dflat.ctypes.data, cap, pid.ctypes.data, gid.ctypes.data,
               pfirst.ctypes.data, gfirst.ctypes.data, nid.ctypes.data, wanted.ctypes.data, rootish.ctypes.data,
               restr.ctypes.data)
        if e <= cap:
            break
        cap = e
    return (cnt, dflat[:e], misses, pid, pfirst[:nid[0]], gid, gfirst[:nid[1]], wanted, rootish, restr)


def _columns_py(tss):
    """_columns_c's result with Python passes (one C-level map per column)."""
    n = len(tss)
    deps = list(map(_DEPS, tss))
    cnt = np.fromiter(map(len, deps), np.int64, n)
    tid = dict(zip(map(id, tss), range(n)))
    flat = list(chain.from_iterable(deps))
    none = -(1 << 40)
    dflat = np.fromiter(map(tid.get, map(id, flat), repeat(none)), np.int64, len(flat))
    misses, mid = [], {}
    for k in np.flatnonzero(dflat == none).tolist():
        d = flat[k]
        m = mid.get(id(d))
        if m is None:
            m = mid[id(d)] = len(misses)
            misses.append(d)
        dflat[k] = -1 - m
    pid, pfirst = _first_seen(list(map(_PREFIX, tss)))
    gid, gfirst = _first_seen(list(map(_GROUP, tss)))
    restr = np.zeros(n, np.uint8)
    for b, get in enumerate(_RESTR):
        restr |= np.fromiter(map(truth, map(get, tss)), np.uint8, n) << b
    return (cnt, dflat, misses, pid, pfirst, gid, gfirst, np.fromiter(map(truth, map(_WANTS, tss)), np.uint8, n),
            np.fromiter(map(_ROOTISH_CODE.__getitem__, map(_ROOTISH, tss)), np.int8, n), restr)


def _first_seen(objs):
    """(ids of ``objs`` in first-seen order, the first position of each id); identity
    hashing (TaskGroup / TaskPrefix define no __hash__)."""
    ids = np.fromiter(map(dict(zip(map(id, reversed(objs)), range(len(objs) - 1, -1, -1))).__getitem__,
                          map(id, objs)), np.int64, len(objs))
    first = np.unique(ids)  # positions of first occurrences, ascending = first-seen order
    rank = np.zeros(len(objs), np.int32)
    rank[first] = np.arange(len(first), dtype=np.int32)
    return rank[ids], first.astype(np.int32)


def graph_from_tasks(tss, nthreads, valid_workers=None, worker_index=None, earlier=None):
    """TaskState objects -> the engine's graph arrays (the layout of distributed_amd/graphs.py).

    Tasks are indexed in ascending ``TaskState.priority`` (so ``prio`` is their rank: unique
    and topological for dask.order priorities); dependencies must be among ``tss`` or, with
    ``earlier`` (key -> engine index of the tasks already uploaded), earlier tasks, which a
    row names as ``-1 - index`` (dgp_add_graph).
    Prefixes / groups get ids in first-seen order; ``prefix_default_dur`` is each
    ``TaskPrefix.duration_average`` now (default-task-durations or -1).

    Restrictions: with ``valid_workers`` (``SchedulerState.valid_workers``, scheduler.py
    :3043-3107, which resolves worker / host / resource restrictions) and ``worker_index``
    (address -> engine worker index), every task with restrictions gets its valid set as
    ascending indices (``restr_ptr`` / ``restr_idx``) and ``restr_flags`` (1: restricted,
    2: loose_restrictions).

    Every per-task column is one C-level pass (``map`` over attribute getters into
    ``np.fromiter``): no Python frame and no container allocation per task (a Python loop
    here costs ~10 us per task, mostly the collector walking the scheduler's heap); only
    restricted tasks and dependencies on earlier graphs are visited one by one. Returns
    (graph, keys in engine order, their priorities)."""
    prio = list(map(_PRIO, tss))
    if not all(map(lt, prio, islice(prio, 1, None))):  # not already in ascending priority
        tss = sorted(tss, key=_PRIO)
        prio = list(map(_PRIO, tss))
    n = len(tss)
    keys = list(map(_KEY, tss))
    fn = _ingest_lib()
    use_c = fn is not None and not _FORCE_PY_INGEST
    cnt, didx, misses, pid, pfirst, gid, gfirst, wanted, rootish, restr = (
        _columns_c(fn, tss) if use_c else _columns_py(tss))
    # a dependency outside the graph: an earlier task (engine index e -> -1 - e), else an error
    none = -(1 << 40)
    if misses:
        eidx = np.fromiter(map((earlier or {}).get, map(_KEY, misses), repeat(none)), np.int64, len(misses))
        lost = np.flatnonzero(eidx == none)
        if len(lost):
            m = int(lost[0])
            k = int(np.flatnonzero(didx == -1 - m)[0])
            row = int(np.searchsorted(np.cumsum(cnt), k, side="right"))
            raise ValueError(f"dependency {misses[m].key!r} of {keys[row]!r} is not in the uploaded graph")
        out = didx < 0
        didx[out] = -1 - eidx[-1 - didx[out]]
    if misses or not use_c:  # each row ascending (one lexsort over the flat edges; the C pass sorted them)
        rowid = np.repeat(np.arange(n, dtype=np.int64), cnt)
        didx = didx[np.lexsort((didx, rowid))]
    prefixes = [tss[i].prefix for i in pfirst.tolist()]
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(cnt, out=ptr[1:])
    g = dict(
        n_tasks=n,
        dep_ptr=ptr,
        dep_idx=didx.astype(np.int32),
        prio=np.arange(n, dtype=np.int64),
        prefix_id=pid,
        group_id=gid,
        prefix_names=[p.name for p in prefixes],
        group_names=[tss[i].group.name for i in gfirst.tolist()],
        group_prefix=pid[gfirst].astype(np.int32),
        prefix_default_dur=np.array([float(p.duration_average) for p in prefixes], np.float64),
        wanted=wanted,
        rootish_override=rootish,
        nthreads=np.asarray(nthreads, np.int32),
        # completion reports arrive with the task-finished messages (service mode)
        nbytes=np.full(n, -1, np.int64),
        start=np.zeros(n),
        stop=np.zeros(n),
    )
    if valid_workers is not None and restr.any():
        flags = np.zeros(n, np.uint8)
        vrows = {}
        for i in np.flatnonzero(restr).tolist():
            ts = tss[i]
            vw = valid_workers(ts)
            if vw is None:  # restrictions that exclude nobody
                continue
            flags[i] = 1 | (2 if ts.loose_restrictions else 0)
            vrows[i] = sorted(worker_index[ws.address] for ws in vw)
        if vrows:
            rc = np.zeros(n, np.int64)
            for i, r in vrows.items():
                rc[i] = len(r)
            rp = np.zeros(n + 1, np.int64)
            np.cumsum(rc, out=rp[1:])
            g.update(restr_ptr=rp, restr_idx=np.array([w for i in sorted(vrows) for w in vrows[i]], np.int32),
                     restr_flags=flags)
    return g, keys, prio


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
        self.prefix_index: dict = {}  # prefix name -> the engine's slot (at most prefixes.PX live at once)
        # every engine task's prefix (an index into pnames, stable for the session), each
        # name's default duration, and the tasks whose device slot is a placeholder since a
        # compaction left their (then dead) prefix out (prefixes.py)
        self.pnames: list = []
        self.pname_id: dict = {}
        self.pname_dur: dict = {}
        self.task_pname = np.zeros(0, np.int32)
        self._stale: set = set()
        self.dev_run: dict = {}   # key -> placement-log position of its current placement
        self.pending: deque = deque()  # (task index, worker index) in placement order
        self.n_fetched = 0
        self.stats = Counter()
        self._recomputed = set()  # earlier tasks a later graph's stimulus recomputed on the device
        self._allowed: list = []  # per running wrapped stimulus: the transitions the engine follows
        self._window = None       # (allowed transitions, keys or None) after a plugin hook's stimulus
        self._expect_replicas: set = set()  # (key, address) replicas the running stimulus adds itself
        # a stimulus the engine does not model: the scheduler decides it, then a resync
        self.suspended = False
        self.suspend_reason = None
        self._host_pl: list = []    # placements the scheduler made meanwhile (dgp_sync_placements rows)
        self._dirty: set = set()    # keys whose state the scheduler changed meanwhile
        self._dirty_all = False
        self._route = 0             # the decide_worker route of the scheduler's current decision
        self.removed: set = set()   # addresses of removed workers (they keep their engine index)
        self._losing = None         # the worker whose loss the engine decided (its replica drops are the engine's)
        self._loss_token = None     # the open remove_worker window: (its transitions, address)
        self._rootish_h: dict = {}  # key -> the _rootish override the engine holds (-1 / 0 / 1)
        self._restr_h: dict = {}    # key -> (restriction flags, valid worker indices) the engine holds
        # key -> (message batch, row): the who_has / nbytes of the compute-task message of an
        # engine placement not yet sent (dgp_task_messages, fetched with the placements)
        self._msg_of: dict = {}
        self.engine_messages = True
        self.n_engine_messages = 0
        # a task-finished batch the device is answering while the reference's handler runs
        # (dgp_tasks_finished_post): its messages, their (key, worker) pairs, and the replica
        # additions seen before the answer came (classified by _settle)
        self.overlap = True
        self._posted = None
        self._posted_pairs = ()
        self._deferred_adds: list = []
        if hasattr(scheduler, "add_plugin"):
            scheduler.add_plugin(self, name=self.name)
        elif isinstance(getattr(scheduler, "plugins", None), dict):  # a bare SchedulerState
            scheduler.plugins[self.name] = self
        self._install()

    # ---------------------------------------------------------------- plumbing
    def _install(self):
        s = self.scheduler
        table = dict(type(s)._TRANSITIONS_TABLE)
        ref_wp = table[("waiting", "processing")]
        ref_qp = table[("queued", "processing")]

        # called as func(sched, key, stimulus_id, **kwargs) (scheduler.py:1955-1958); a
        # partial is one Python frame less per decision than a closure
        table[("waiting", "processing")] = functools.partial(self._transition_waiting_processing, ref=ref_wp)
        table[("queued", "processing")] = functools.partial(self._transition_queued_processing, ref=ref_qp)
        s._TRANSITIONS_TABLE = table  # per instance: the class table stays untouched
        if not getattr(s, "_gpu_placement_add", False):
            ref_add = s._add_to_processing

            def add_to_processing(ts, ws, stimulus_id):
                if self.suspended and self.active and ts.key in self.task_index and ws.address in self.worker_index:
                    self._host_pl.append((self.task_index[ts.key], self.worker_index[ws.address])
                                         + sync.placement_record(s, ts, ws, self._route))
                return ref_add(ts, ws, stimulus_id=stimulus_id)

            s._add_to_processing = add_to_processing
            s._gpu_placement_add = True
        if not getattr(s, "_gpu_placement_msg", False) and callable(getattr(s, "_task_to_msg", None)):
            ref_msg = s._task_to_msg

            def task_to_msg(ts, duration=-1):
                if self._posted is not None:
                    self._settle()
                m = self._msg_of.pop(ts.key, None)
                if m is None or not self.active:
                    return ref_msg(ts, duration)
                return self._engine_task_msg(ts, duration, *m)

            s._task_to_msg = task_to_msg
            s._gpu_placement_msg = True
        if callable(getattr(s, "handle_stream", None)) and not getattr(s, "_gpu_placement_stream", False):
            s.handle_stream = self.handle_stream  # per instance: Server.handle_stream stays untouched
            s._gpu_placement_stream = True
        handlers = getattr(s, "stream_handlers", None)
        if handlers is not None:
            handlers["task-finished"] = self.handle_task_finished
            # worker stream handlers (scheduler.py:3768-3779); the transitions each may run
            # that the engine follows itself (anything else ends GPU placement)
            self._wrap(handlers, "add-keys", self._on_add_keys, ())
            self._wrap(handlers, "release-worker-data", None, ())
            self._wrap(handlers, "long-running", self._on_long_running, _REFILL_TRANSITIONS)
            self._wrap(handlers, "worker-status-change", self._on_worker_status_change, _REFILL_TRANSITIONS)
            self._wrap(handlers, "task-erred", self._on_task_erred, _ERRED_TRANSITIONS | _RESCHEDULE_TRANSITIONS)
            self._wrap(handlers, "reschedule", self._on_reschedule, _RESCHEDULE_TRANSITIONS)
            # client stream handlers (:3781-3792)
            self._wrap(handlers, "client-desires-keys", self._on_client_desires_keys, ())
            # Scheduler.client_releases_keys per instance, from any caller: the stream handler,
            # stimulus_cancel (cancel-keys :5364-5396, once per cancelled dependent level and
            # client) and remove_client (close-client :5727-5750) -- each call one stimulus
            rel = {"m": getattr(s, "client_releases_keys", None)}
            self._wrap(rel, "m", self._on_client_releases_keys, _RELEASE_TRANSITIONS)
            if rel["m"] is not None:
                s.client_releases_keys = rel["m"]
                handlers["client-releases-keys"] = rel["m"]
            self._wrap(handlers, "cancel-keys", None, ())
            self._wrap(handlers, "close-client", None, ())
            self._wrap(handlers, "update-data", self._on_update_data, ())
        rpc = getattr(s, "handlers", None)
        if isinstance(rpc, dict):
            self._wrap(rpc, "heartbeat_worker", self._on_heartbeat, (), after=True)
        self._wrap_set_restrictions()
        self._wrap_shuffle()
        self._wrap_replicas()
        self._wrap_stealing()
        self._wrap_remove_worker()

    def _wrap(self, table, name, on_event, modelled, after=False):
        """Route stream / RPC handler ``name`` through the extension: ``on_event(kwargs)``
        (before the handler; with ``after`` it gets a callable that runs the handler)
        brings the engine up to date or falls back; the handler itself then runs with
        ``modelled`` as the transitions the engine follows for it (the plugin hook)."""
        orig = table.get(name)
        if orig is None or getattr(orig, "_gpu_placement", False):
            return
        modelled = frozenset(modelled)

        def enter(kwargs):
            self._enter()
            if on_event is not None and self.active and self.engine is not None:
                try:
                    on_event(kwargs)
                except Exception as e:  # an engine failure ends GPU placement, never the scheduler
                    self.fallback(f"{name}: {e}")
            self._allowed.append(modelled)

        def leave():
            self._allowed.pop()
            if self.suspended:
                self._resync()
            self._end_of_stimulus(name)

        if inspect.iscoroutinefunction(orig):
            @functools.wraps(orig)
            async def wrapped(*args, **kwargs):
                enter(kwargs)
                try:
                    return await orig(*args, **kwargs)
                finally:
                    leave()
        elif after:
            @functools.wraps(orig)
            def wrapped(*args, **kwargs):
                self._enter()
                box = {}

                def run():
                    self._allowed.append(modelled)
                    try:
                        box["r"] = orig(*args, **kwargs)
                    finally:
                        self._allowed.pop()
                    return box["r"]

                if on_event is not None and self.active and self.engine is not None:
                    try:
                        on_event(kwargs, run)
                    except Exception as e:
                        self.fallback(f"{name}: {e}")
                r = box["r"] if "r" in box else run()
                if self.suspended:
                    self._resync()
                self._end_of_stimulus(name)
                return r
        else:
            @functools.wraps(orig)
            def wrapped(*args, **kwargs):
                enter(kwargs)
                try:
                    return orig(*args, **kwargs)
                finally:
                    leave()
        wrapped._gpu_placement = True
        table[name] = wrapped

    def _wrap_remove_worker(self):
        """``Scheduler.remove_worker`` (scheduler.py:5180-5362), from any caller (the
        "unregister" RPC, heartbeat timeouts, retire_workers, close_worker): when the worker
        still has processing tasks or sole replicas, the whole stimulus -- its processing
        tasks released and re-placed, its lost results recomputed -- is the engine's
        (dgp_lose_worker, ``_lose_worker``) before the scheduler's own code runs; its
        transitions then take the engine's decisions (validated like any other). A loss the
        engine does not restate keeps the old path: the scheduler decides, then a resync."""
        s = self.scheduler
        orig = getattr(s, "remove_worker", None)
        if orig is None or getattr(orig, "_gpu_placement", False) or not inspect.iscoroutinefunction(orig):
            return

        @functools.wraps(orig)
        async def remove_worker(*args, **kwargs):
            self._enter()
            address = args[0] if args else kwargs.get("address")
            lost = False
            # the reference returns "already-removed" before any transition when the scheduler
            # is closed or the (coerced) address is not a worker (:5193-5199): no engine call then
            live = self._removable(address)
            if live is not None and self.active and self.engine is not None:
                try:
                    lost = self._lose_worker(live, bool(kwargs.get("safe", False)))
                except Exception as e:  # an engine failure ends GPU placement, never the scheduler
                    self.fallback(f"remove_worker({address}): {e}")
            # the loss window closes in the plugin hook (``remove_worker`` below), which the
            # reference calls synchronously right after its transitions (:5298-5317), not across
            # the await of the plugins' awaitables that follows
            token = (_LOSS_TRANSITIONS if lost else frozenset(), live)
            self._loss_token = token
            self._allowed.append(token[0])
            try:
                return await orig(*args, **kwargs)
            finally:
                self._close_loss(token)

        remove_worker._gpu_placement = True
        s.remove_worker = remove_worker  # per instance: every self.remove_worker call goes through it
        rpc = getattr(s, "handlers", None)
        if isinstance(rpc, dict) and "unregister" in rpc:
            rpc["unregister"] = remove_worker

    def _removable(self, address):
        """The address ``Scheduler.remove_worker`` would act on, or None when it returns
        "already-removed" without a transition (scheduler closed, not a worker)."""
        s = self.scheduler
        st = getattr(s, "status", None)
        if getattr(st, "name", st) == "closed":
            return None
        coerce = getattr(s, "coerce_address", None)
        if callable(coerce):
            try:
                address = coerce(address)
            except Exception:
                return None
        return address if address in getattr(s, "workers", {}) else None

    def _close_loss(self, token):
        """End the window a ``remove_worker`` stimulus opened (once: the plugin hook or,
        when the reference returned early, the wrapper's ``finally``)."""
        if getattr(self, "_loss_token", None) is not token:
            return
        self._loss_token = None
        if self._allowed and self._allowed[-1] is token[0]:
            self._allowed.pop()
        self._losing = None

    def _lose_worker(self, address, safe) -> bool:
        """The engine's half of a worker loss (see ``_wrap_remove_worker``): True when the
        engine decided the stimulus (its placements are queued for the transitions)."""
        s = self.scheduler
        ws = s.workers.get(address)
        if ws is None or address not in self.worker_index or self.suspended:
            return False
        if not hasattr(self.engine, "lose_worker"):
            return False
        proc, held = list(ws.processing), list(ws.has_what)  # the orders remove_worker iterates (:5236, :5270)
        if not proc and not any(ts.who_has == {ws} for ts in held):
            return False  # a drained worker: no transition (the plugin hook follows it)
        ti = self.task_index
        plan = None
        if not (any(ts.key not in ti for ts in proc) or any(ts.who_has == {ws} and ts.key not in ti for ts in held)):
            plan = loss.supported(s, ws, proc, held, safe)
        # every task the cascade may re-wait, place or err is the engine's, with its prefix's slot
        if plan is None or any(ts.key not in ti or ts.prefix.name not in self.prefix_index or ti[ts.key] in self._stale
                               for ts in plan[0] + plan[1] + loss.lost_results(ws, held)):
            self.stats["losses_left_to_scheduler"] += 1
            return False
        self._end_of_stimulus("the previous stimulus")
        if not self.active:
            return False
        chain, erred = plan
        killed = loss.killed_flags(s, proc, safe)
        order = loss.loss_orders(chain, lambda ts: ti[ts.key], erred, sum(killed))
        n = self.engine.lose_worker(self.worker_index[address], [ti[ts.key] for ts in proc],
                                    [ti[ts.key] for ts in held if ts.key in ti], order, killed)
        if n is None:  # refused: the scheduler decides, the engine resyncs after
            self._suspend(f"remove_worker({address}): {getattr(self.engine, 'refusal', 'refused by the engine')}")
            return False
        self._losing = address
        self.stats["workers_lost_on_device"] += 1
        self._fetch(n)
        return True

    def _wrap_replicas(self):
        """``SchedulerState.add_replica`` / ``remove_replica`` (scheduler.py:3148-3159) from
        any caller (add-keys :7375, a task-finished for a task already in memory :5082,
        release-worker-data :5813, update_data :7416, rebalance / replicate :6454, :6493):
        who_has and ws.nbytes are inputs of decide_worker / worker_objective
        (:8571-8593, :3131-3146). The completing task's own replica (_add_to_memory :3296)
        is part of the task-finished stimulus the engine runs."""
        s = self.scheduler
        if getattr(s, "_gpu_placement_replicas", False):
            return
        add0, rem0 = s.add_replica, s.remove_replica

        def add_replica(ts, ws):
            k = (ts.key, ws.address)
            if self._posted is not None:
                if k in self._posted_pairs:  # the batch's own completion: classified by the answer
                    self._deferred_adds.append((ts, ws, ws in (ts.who_has or ())))
                    return add0(ts, ws)
                self._settle()
            if k in self._expect_replicas:
                self._expect_replicas.discard(k)
            elif ws not in (ts.who_has or ()):
                self._replica_event(ts, ws, +1)
            return add0(ts, ws)

        def remove_replica(ts, ws):
            if self._posted is not None:
                self._settle()
            if ws in (ts.who_has or ()):
                self._replica_event(ts, ws, -1)
            return rem0(ts, ws)

        s.add_replica = add_replica
        s.remove_replica = remove_replica
        s._gpu_placement_replicas = True

    def _wrap_set_restrictions(self):
        """``Scheduler.set_restrictions`` (scheduler.py:7702-7707), both as the RPC handler
        and as the method other extensions call -- the P2P shuffle's ``restrict_task`` ->
        ``_set_restriction`` (shuffle/_scheduler_plugin.py:101-115, :281-293) calls
        ``self.scheduler.set_restrictions``: a task's valid workers change outside any
        transition, which the engine takes over (``dgp_update_restrictions``)."""
        s = self.scheduler
        orig = getattr(s, "set_restrictions", None)
        if orig is None or getattr(orig, "_gpu_placement", False):
            return

        @functools.wraps(orig)
        def set_restrictions(*args, **kwargs):
            worker = kwargs["worker"] if "worker" in kwargs else (args[0] if args else {})
            r = orig(*args, **kwargs)
            self._task_inputs_changed(list(worker or {}))
            return r

        set_restrictions._gpu_placement = True
        s.set_restrictions = set_restrictions  # per instance: other extensions call it through self
        rpc = getattr(s, "handlers", None)
        if isinstance(rpc, dict) and "set_restrictions" in rpc:
            rpc["set_restrictions"] = set_restrictions

    def _wrap_shuffle(self):
        """The P2P shuffle plugin (shuffle/_scheduler_plugin.py) sets ``_rootish = False`` on
        the barrier's dependents by plain attribute assignment when a shuffle starts
        (``_ensure_output_tasks_are_non_rootish`` :150-151, :254-278): the engine takes the new
        overrides after it (``dgp_set_rootish``)."""
        s = self.scheduler
        sh = (getattr(s, "extensions", None) or {}).get("shuffle")
        fn = getattr(sh, "_ensure_output_tasks_are_non_rootish", None)
        if fn is None or getattr(fn, "_gpu_placement", False):
            return

        @functools.wraps(fn)
        def ensure_non_rootish(spec, *args, **kwargs):
            r = fn(spec, *args, **kwargs)
            try:
                from distributed.shuffle._core import barrier_key

                barrier = s.tasks.get(barrier_key(spec.id))
                keys = [d.key for d in barrier.dependents] if barrier is not None else list(self.task_index)
            except Exception:  # no barrier name: every task the engine holds
                keys = list(self.task_index)
            self._task_inputs_changed(keys)
            return r

        ensure_non_rootish._gpu_placement = True
        sh._ensure_output_tasks_are_non_rootish = ensure_non_rootish

    def _task_rows(self, ts):
        """(_rootish override, restriction flags, valid worker indices) of ``ts`` as the
        engine holds them (graph_from_tasks' resolution, valid_workers :3043-3107)."""
        ov = -1 if ts._rootish is None else int(bool(ts._rootish))
        if ts.worker_restrictions or ts.host_restrictions or ts.resource_restrictions:
            vw = self.scheduler.valid_workers(ts)
            if vw is not None:
                row = tuple(sorted(self.worker_index[ws.address] for ws in vw if ws.address in self.worker_index))
                return ov, 1 | (2 if ts.loose_restrictions else 0), row
        return ov, 0, ()

    def _task_inputs_changed(self, keys):
        """TaskState._rootish / restrictions of ``keys`` may have changed outside any
        transition: the engine takes the differences from what it holds. Under a suspension
        the keys are marked dirty instead (the resync takes them)."""
        if not self.active or self.engine is None:
            return
        keys = [k for k in keys if k in self.task_index]
        if not keys:
            return
        if self.suspended:
            self._dirty.update(keys)
            return
        self._push_task_inputs(keys)

    def _push_task_inputs(self, keys):
        s = self.scheduler
        rt, rv, ut, urows, uflags = [], [], [], [], []
        for k in keys:
            ts = s.tasks.get(k)
            if ts is None:
                continue
            t = self.task_index[k]
            ov, fl, row = self._task_rows(ts)
            if ov != self._rootish_h.get(k, -1):
                rt.append(t)
                rv.append(ov)
                self._rootish_h[k] = ov
            if (fl, row) != self._restr_h.get(k, (0, ())):
                ut.append(t)
                urows.append(row)
                uflags.append(fl)
                self._restr_h[k] = (fl, row)
        if rt:
            self._engine_op("set_rootish", rt, rv)
        if ut:
            self._engine_op("update_restrictions", ut, urows, uflags)

    def _replica_event(self, ts, ws, sign):
        if not self.active or self.engine is None or ts.key not in self.task_index:
            return
        if self.suspended:  # the resync carries it
            self._dirty.add(ts.key)
            return
        if sign < 0 and ws.address == self._losing:  # dgp_lose_worker dropped the lost worker's replicas
            return
        w = self.worker_index.get(ws.address)
        what = "add_replicas" if sign > 0 else "remove_replicas"
        if w is None:
            self._suspend(f"{what}({ts.key!r}, {ws.address}): worker not in the engine's table")
            self._dirty.add(ts.key)
            return
        if sign < 0 and len(ts.who_has or ()) <= 1:
            # the last replica: release-worker-data recomputes the task (:5813-5815)
            self._suspend(f"the last replica of {ts.key!r} leaves {ws.address}")
            self._dirty.add(ts.key)
            return
        self._engine_op(what, [self.task_index[ts.key]], [w])

    def _engine_op(self, what, *args):
        """Follow one placement-input change on the device; an engine without that
        operation (or one that fails) hands placement back to the scheduler."""
        if self._posted is not None:
            self._settle()
        fn = getattr(self.engine, what, None)
        if fn is None:
            self.fallback(f"{what}: not modelled by the engine")
            return None
        self._end_of_stimulus("the previous stimulus")
        if not self.active:
            return None
        try:
            r = fn(*args)
        except Exception as e:
            if "does not model" in str(e):  # refused, nothing changed on the device
                self._suspend(f"{what}: {e}")
            else:
                self.fallback(f"{what}: {e}")
            return None
        self.stats[what] += 1
        self._fetch()  # a refill the operation made (resume, long-running)
        return r

    def _wrap_stealing(self):
        """Follow the stealing extension (stealing.py). ``move_task_confirm`` (:333-399, also
        its ``steal-response`` stream handler :121): a confirmed steal moves the task on the
        engine (``dgp_move_task``); the finally clause's check_idle_saturated of thief and
        victim (:396-399) and ``balance``'s check_idle_saturated(victim, occ=combined
        occupancy) (:494-496) change idle / saturated membership outside any placement,
        which the engine takes over (``set_worker_flags``)."""
        s = self.scheduler
        st = (getattr(s, "extensions", None) or {}).get("stealing")
        if st is None or getattr(st, "_gpu_placement_wrapped", False):
            return
        orig = st.move_task_confirm

        async def move_task_confirm(*, key, state, stimulus_id, worker=None):
            # a stimulus of its own: a resync the previous one left pending runs first (the
            # engine refuses a move while it waits for one)
            self._enter()
            ts = s.tasks.get(key)
            before = ts.processing_on if ts is not None and ts.state == "processing" else None
            flags0 = self._flags_of(s)
            try:
                await orig(key=key, state=state, stimulus_id=stimulus_id, worker=worker)
            finally:
                ts = s.tasks.get(key)
                moved = False
                if before is not None and ts is not None:
                    if ts.state == "processing" and ts.processing_on is not None and ts.processing_on is not before:
                        self.task_moved(ts, ts.processing_on)
                        moved = True
                    elif ts.state != "processing":  # "reschedule" (:365-376): not modelled on the device
                        self.fallback(f"steal of {key!r} rescheduled it")
                if not moved:  # the reject branches re-check thief and victim (:396-399)
                    self._sync_flags(flags0)

        st.move_task_confirm = move_task_confirm
        if getattr(s, "stream_handlers", None) is not None and "steal-response" in s.stream_handlers:
            s.stream_handlers["steal-response"] = move_task_confirm
        bal = getattr(st, "balance", None)
        if bal is not None:
            @functools.wraps(bal)
            def balance(*args, **kwargs):
                self._enter()  # a periodic callback: its own stimulus (a pending resync first)
                flags0 = self._flags_of(s)
                try:
                    return bal(*args, **kwargs)
                finally:
                    self._sync_flags(flags0)

            st.balance = balance
            pcs = getattr(s, "periodic_callbacks", None) or {}
            pc = pcs.get("stealing")
            if pc is not None and getattr(pc, "callback", None) is bal:
                pc.callback = balance
        st._gpu_placement_wrapped = True

    @staticmethod
    def _flags_of(s):
        return set(getattr(s, "idle", {}) or {}), {ws.address for ws in (getattr(s, "saturated", ()) or ())}

    def _sync_flags(self, before):
        """Idle / saturated membership the scheduler changed outside a placement: the
        engine's worker flags take the scheduler's (``set_worker_flags``)."""
        if not self.active or self.engine is None:
            return
        s = self.scheduler
        idle1, sat1 = self._flags_of(s)
        idle0, sat0 = before
        changed = sorted((idle0 ^ idle1) | (sat0 ^ sat1))
        if not changed:
            return
        if any(a not in self.worker_index for a in changed):
            self.fallback("idle / saturated change of a worker not in the engine's table")
            return
        self._engine_op("set_worker_flags", [self.worker_index[a] for a in changed],
                        [1 if a in idle1 else 0 for a in changed], [1 if a in sat1 else 0 for a in changed])

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

    def _enter(self):
        """A new stimulus starts: the previous one's window closes and, if the scheduler
        decided it itself, the engine takes the scheduler's state first."""
        self._close_window()
        if self.suspended:
            self._resync()

    def _suspend(self, reason: str):
        """The running stimulus is the scheduler's own (a change the engine does not model):
        its remaining decisions come from the scheduler's Python and the engine resynchronises
        from the scheduler's state when it ends (dgp_sync_*). An engine without the resync
        entry points hands placement back for good (``fallback``)."""
        if not self.active or self.engine is None:
            return
        if not all(hasattr(self.engine, m) for m in ("sync_placements", "sync_tasks", "sync_workers",
                                                       "sync_globals")):
            self.fallback(reason)
            return
        if not self.suspended:
            logger.info("gpu-placement: the scheduler decides this stimulus, then the engine resynchronises: %s", reason)
            self.suspended = True
            self.suspend_reason = reason
            self._host_pl = []
            self.pending.clear()
            self.stats["suspended"] += 1

    def _mark_dirty(self, key):
        """A task whose state changed under suspension, and the neighbours whose waiting_on /
        waiters counts it moves."""
        self._dirty.add(key)
        ts = self.scheduler.tasks.get(key)
        if ts is not None:
            self._dirty.update(d.key for d in ts.dependencies)
            self._dirty.update(d.key for d in ts.dependents)

    def _resync(self):
        """dgp_sync_placements / _tasks / _workers / _globals from the scheduler's state."""
        s = self.scheduler
        try:
            pl = self._host_pl
            cols = list(zip(*pl)) if pl else [[]] * 6
            placements = dict(zip(("task", "worker", "comm", "start", "wsnbytes", "route"), cols))
            keys = self.keys if self._dirty_all else [k for k in self._dirty if k in self.task_index]
            if hasattr(self.engine, "remap_prefixes") and not self._prefixes_current(keys):
                self._compact_prefixes([], resync=False)  # the rows below come in the new numbering
            widx = {a: i for i, a in enumerate(self.workers)}
            tasks = sync.task_rows(s, keys, self.task_index, widx)
            workers = sync.worker_rows(s, self.workers, self.prefix_index, self.task_index)
            pnames = sorted(self.prefix_index, key=self.prefix_index.get)
            gnames = sorted(self.group_index, key=self.group_index.get)
            glob = sync.global_rows(s, pnames, self.prefix_dur, gnames, self.task_index, widx)
            n0 = self.engine.num_placements()
            self.engine.sync(placements, tasks, workers, glob)
            for j, p in enumerate(pl):
                self.dev_run[self.keys[p[0]]] = n0 + j
            self.n_fetched = self.engine.num_placements()
            # _rootish / restrictions the scheduler changed meanwhile (set_restrictions, the
            # shuffle's restrict_task, _ensure_output_tasks_are_non_rootish, a later graph's)
            self.suspended = False
            self._push_task_inputs(keys)
            self.stats["resyncs"] += 1
            self.stats["resync_tasks"] += len(keys)
        except Exception as e:
            self.fallback(f"resync after '{self.suspend_reason}': {e}")
        self.suspended = False
        self._host_pl = []
        self._dirty = set()
        self._dirty_all = False
        self.pending.clear()

    def _config(self):
        from distributed import scheduler as sched_mod

        s = self.scheduler
        sat = s.WORKER_SATURATION
        return {"bandwidth": int(s.bandwidth), "default_data_size": int(sched_mod.DEFAULT_DATA_SIZE),
                "unknown_duration": float(s.UNKNOWN_TASK_DURATION),
                "saturation": "inf" if math.isinf(sat) else float(sat)}

    def _fetch(self, n_new=None, messages=True):
        """Queue the engine's new placements (the decisions the transitions will ask for);
        ``n_new``: how many the last engine call reported (saves a device round trip).
        ``messages``: also take their compute-task messages' who_has / nbytes from the
        engine (dgp_task_messages: its replica state after the call, which is the state each
        message is built in when the call was one stimulus, or several whose later members
        add no replica of an earlier one's dependencies)."""
        n = self.engine.num_placements() if n_new is None else self.n_fetched + n_new
        if n > self.n_fetched:
            n0 = self.n_fetched
            want = messages and self.engine_messages and hasattr(self.engine, "task_messages")
            if hasattr(self.engine, "answer"):  # one call, preallocated buffers
                tasks, workers, batch = self.engine.answer(n0, n - n0, want)
            else:
                pl = self.engine.placements(n0, n - n0, columns=("pl_task", "pl_worker"))
                tasks, workers, batch = pl["pl_task"].tolist(), pl["pl_worker"].tolist(), None
                if want:
                    m = self.engine.task_messages(n0, n - n0)
                    batch = tuple(m[k].tolist() for k in ("dep_ptr", "dep_task", "dep_nbytes", "holder_ptr",
                                                          "holder_idx"))
            keys, dev_run, pending = self.keys, self.dev_run, self.pending
            j = n0
            for t, w in zip(tasks, workers):
                pending.append((t, w))
                dev_run[keys[t]] = j
                j += 1
            self.n_fetched = n
            if batch is not None:
                msg_of = self._msg_of
                for i, t in enumerate(tasks):
                    msg_of[keys[t]] = (batch, i)

    def _engine_task_msg(self, ts, duration, batch, i):
        """``SchedulerState._task_to_msg`` (scheduler.py:3421-3450) for a placement the engine
        made, its ``who_has`` / ``nbytes`` from the engine's batch (dgp_task_messages: the
        dependencies in CSR order, their holders ascending by worker index) instead of a
        walk over the dependencies' replica sets; every other field as there."""
        sm = _SM or _sched_mod()
        dep_ptr, dep_task, dep_nbytes, holder_ptr, holder_idx = batch
        keys, addrs = self.keys, self.workers
        who_has, nbytes = {}, {}
        d0, d1 = dep_ptr[i], dep_ptr[i + 1]
        for k in range(d0, d1) if d1 > d0 else ():
            dk = keys[dep_task[k]]
            h0, h1 = holder_ptr[k], holder_ptr[k + 1]
            who_has[dk] = [addrs[holder_idx[h0]]] if h1 == h0 + 1 else [addrs[h] for h in holder_idx[h0:h1]]
            nbytes[dk] = dep_nbytes[k]
        if self.validate:
            ref_who = {d.key: sorted(ws.address for ws in d.who_has or ()) for d in ts.dependencies}
            ref_nb = {d.key: d.nbytes for d in ts.dependencies}
            if {k: sorted(v) for k, v in who_has.items()} != ref_who or nbytes != ref_nb:
                raise AssertionError(f"gpu-placement: compute-task message of {ts.key!r}: engine who_has "
                                     f"{who_has} nbytes {nbytes}, the reference {ref_who} {ref_nb}")
        if duration < 0:
            duration = self.scheduler.get_task_duration(ts)
        ts.run_id = next(sm.TaskState._run_id_iterator)
        assert ts.priority, ts
        self.n_engine_messages += 1
        return {
            "op": "compute-task",
            "key": ts.key,
            "run_id": ts.run_id,
            "priority": ts.priority,
            "duration": duration,
            "stimulus_id": f"compute-task-{sm.time()}",
            "who_has": who_has,
            "nbytes": nbytes,
            "run_spec": sm.ToPickle(ts.run_spec),
            "resource_restrictions": ts.resource_restrictions,
            "actor": ts.actor,
            "annotations": ts.annotations or {},
            "span_id": ts.group.span_id,
        }

    def _end_of_stimulus(self, what: str):
        if self._posted is not None:
            self._settle()
        self._msg_of.clear()
        if self.active and self.pending:
            t, w = self.pending[0]
            self.fallback(f"{what}: the engine placed {self.keys[t]!r} on {self.workers[w]} but the scheduler "
                          "did not ask for it")

    def _close_window(self):
        self._window = None

    # ------------------------------------------------------- placement decisions
    def _decision(self, sched, ts, queued: bool):
        """The engine's worker for ``ts`` (a WorkerState), None (the engine did not place
        it in this stimulus: it stays / goes queued), or _REF (run the reference)."""
        if self._posted is not None:  # the batch's answer, which the device computed meanwhile
            self._settle()
        if not self.active or self.engine is None:
            return _REF
        if self.suspended:
            self._route = self._route_of(sched, ts, queued)
            return _REF
        pending = self.pending
        if pending and self.keys[pending[0][0]] == ts.key:  # the common case: the engine's next placement
            _, w = pending.popleft()
            self.stats["device_decisions"] += 1
            return sched.workers[self.workers[w]]
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
        # not placed by the engine: only a root-ish task under queuing may stay / go queued,
        # and only when decide_worker_rootish_queuing_enabled finds no slot, i.e.
        # idle_task_count is empty (:2227-2229); anything else is a stimulus the engine did
        # not run (a refill after a change it never saw)
        if queued or (not math.isinf(sched.WORKER_SATURATION) and sched.is_rootish(ts)):
            if sched.idle_task_count:
                self.fallback(f"the scheduler has an open slot for queued {ts.key!r} but the engine left it queued")
                return _REF
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

    @staticmethod
    def _route_of(sched, ts, queued: bool) -> int:
        """The decide_worker route the scheduler's own decision takes (include/dgplace.h
        DGP_ROUTE_*; the routes of tests/golden/gen_golden.py)."""
        if queued:
            return 1
        if sched.is_rootish(ts):
            return 2 if math.isinf(sched.WORKER_SATURATION) else 1
        if ts.dependencies or sched.valid_workers(ts) is not None or len(sched.running) < len(sched.workers):
            return 0
        return 3

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

    def _transition_waiting_processing(self, sched, key, stimulus_id, ref=None, **kwargs):
        """_transition_waiting_processing (scheduler.py:2313-2336) with the engine's decision."""
        ts = sched.tasks[key]
        ws = self._decision(sched, ts, False)
        if ws is _REF:
            return ref(sched, key, stimulus_id)
        if self.validate:
            self._check(sched, ts, ws, False)
        if ws is None:
            if sched.is_rootish(ts) and not math.isinf(sched.WORKER_SATURATION):
                return {ts.key: "queued"}, {}, {}
            return {ts.key: "no-worker"}, {}, {}
        return sched._add_to_processing(ts, ws, stimulus_id=stimulus_id)

    def _transition_queued_processing(self, sched, key, stimulus_id, ref=None, **kwargs):
        """_transition_queued_processing (scheduler.py:2797-2808) with the engine's decision."""
        ts = sched.tasks[key]
        ws = self._decision(sched, ts, True)
        if ws is _REF:
            return ref(sched, key, stimulus_id)
        if self.validate:
            self._check(sched, ts, ws, True)
        if ws is None:
            return {}, {}, {}
        sched.queued.discard(ts)
        return sched._add_to_processing(ts, ws, stimulus_id=stimulus_id)

    # ----------------------------------------------------------- plugin hooks
    def transition(self, key, start, finish, *args, stimulus_id=None, **kwargs):
        """SchedulerPlugin.transition (diagnostics/plugin.py:111-139), called after every
        transition (scheduler.py:2013-2027): the catch-all. A transition outside the
        stimuli the engine follows, or of a kind it does not model, means the scheduler's
        state moved where the engine's did not."""
        pair = (start, finish)
        if self._allowed and pair in self._allowed[-1] and not self.suspended:  # the stimulus' own, followed
            return
        if not self.active or self.engine is None:
            return
        if start == finish:  # a decision that only recommends (queued / no-worker next): no change
            return
        if self._posted is not None:
            self._settle()
            if not self.active:
                return
        w = self._window
        if w is not None and pair in w[0] and (w[1] is None or key in w[1]):
            return
        if key not in self.task_index:
            return  # a task the engine does not hold (scattered data, a graph it did not take)
        if not self.suspended:
            self._suspend(f"transition {start} -> {finish} of {key!r} (stimulus {stimulus_id}) is not modelled "
                          "by the engine")
        self._mark_dirty(key)

    def update_graph(self, scheduler, *, client=None, keys=(), tasks=(), annotations=None, priority=None,
                     dependencies=None, **kwargs):
        """SchedulerPlugin.update_graph (diagnostics/plugin.py:74-109): runs before the
        scheduler transitions the new tasks (scheduler.py:4641-4653)."""
        self._enter()
        if not self.active:
            return
        s = self.scheduler
        # Scheduler.update_graph fills ``priority`` in descending TaskState.priority
        # (scheduler.py:4601-4611): reversed, the tasks arrive in engine order
        try:
            new = list(map(s.tasks.__getitem__, reversed(priority or {})))
        except KeyError:  # a key the scheduler no longer holds
            new = [ts for ts in map(s.tasks.get, reversed(priority or {})) if ts is not None]
        if self.task_index:
            ti = self.task_index
            new = [ts for ts in new if ts.key not in ti]
        if not new:
            return
        try:
            if self.engine is not None:
                keys_ = self._add_graph(new)
            else:
                self.workers = list(s.workers)
                self.worker_index = {a: i for i, a in enumerate(self.workers)}
                if any(ws.status.name != "running" for ws in s.workers.values()):
                    raise NotImplementedError("a worker is not running at the first graph")
                g, keys_, prio_ = graph_from_tasks(new, [s.workers[a].nthreads for a in self.workers],
                                                   s.valid_workers, self.worker_index)
                self.keys = keys_
                self.task_index = dict(zip(keys_, range(len(keys_))))
                self._remember_inputs(g, keys_)
                self.prefix_index = {nm: i for i, nm in enumerate(g["prefix_names"])}
                self.group_index = {nm: i for i, nm in enumerate(g["group_names"])}
                self.prefix_dur = list(g["prefix_default_dur"])
                self._note_prefixes(g)
                self.group_prefix = list(g["group_prefix"])
                self.max_priority = prio_[-1]
                self.prio_of = prio_  # engine index -> TaskState.priority
                if self.engine_factory is not None:
                    self.engine = self.engine_factory()
                else:
                    from .engine import PlacementEngine

                    self.engine = PlacementEngine(self.device)
                self.engine.load(g, self._config(), results=False)
                # task-finished batches through the resident kernel (dgp_set_resident): no
                # launch / copy / sync per call; every other engine call ends it first
                self.engine.set_resident(True)
                if self.engine_messages and hasattr(self.engine, "set_task_messages"):
                    # ... and their answers carry the compute-task message fields (f3)
                    self.engine.set_task_messages(True)
                self.engine.update_graph()
                self._fetch()
                self.stats["graphs"] += 1
            if self.active and keys_ is not None:  # the first graph's keys: the index's key view
                # (a later graph's stimulus that recomputed earlier tasks: theirs too)
                self._window = (_UPDATE_GRAPH_TRANSITIONS,
                                self.task_index.keys() if len(keys_) == len(self.task_index)
                                else set(keys_) | self._recomputed)
            self._recomputed = set()
        except Exception as e:  # plugin errors are logged, not raised (scheduler.py:4652-4653)
            self.fallback(f"update_graph: {e}")

    def _note_prefixes(self, g):
        """Each new engine task's prefix name (session-stable ids) and the names' defaults."""
        ids = []
        for nm, d in zip(g["prefix_names"], g["prefix_default_dur"]):
            if nm not in self.pname_id:
                self.pname_id[nm] = len(self.pnames)
                self.pnames.append(nm)
                self.pname_dur[nm] = float(d)
            ids.append(self.pname_id[nm])
        lut = np.array(ids or [0], np.int32)
        self.task_pname = np.concatenate([self.task_pname, lut[np.asarray(g["prefix_id"], np.int64)]]).astype(np.int32)

    def _compact_prefixes(self, extra, resync: bool):
        """The engine's prefix table compacted to the live prefixes + ``extra``
        (prefixes.py): dgp_remap_prefixes, then (``resync``) the workers' and global rows in
        the new numbering; otherwise the caller's resync follows."""
        s = self.scheduler
        table = prefixes.compacted(self.prefix_index, prefixes.live_prefixes(s), extra)
        if table is None:
            raise NotImplementedError(f"more than {prefixes.PX} live task prefixes")
        old_names = sorted(self.prefix_index, key=self.prefix_index.get)
        slots, stale = prefixes.task_slots(self.task_pname, self.pnames, table)
        names = sorted(table, key=table.get)
        defaults = [self.pname_dur.get(nm, -1.0) for nm in names]
        self.engine.remap_prefixes(slots, defaults)
        self.prefix_index = table
        self.prefix_dur = defaults
        self.group_prefix = [table.get(old_names[p], 0) if 0 <= p < len(old_names) else 0 for p in self.group_prefix]
        self._stale = set(stale.tolist())
        self.stats["prefix_compactions"] += 1
        if resync:
            widx = {a: i for i, a in enumerate(self.workers)}
            workers = sync.worker_rows(s, self.workers, self.prefix_index, self.task_index)
            gnames = sorted(self.group_index, key=self.group_index.get)
            glob = sync.global_rows(s, names, self.prefix_dur, gnames, self.task_index, widx)
            self.engine.sync(None, None, workers, glob)

    def _prefixes_current(self, keys) -> bool:
        """Every live prefix has a slot and no live task among ``keys`` (the resync's) holds a
        placeholder slot (its prefix was dead at a compaction, then recomputed)."""
        s = self.scheduler
        if not set(prefixes.live_prefixes(s)) <= set(self.prefix_index):
            return False
        if self._stale:
            ti = self.task_index
            for k in keys:
                ts = s.tasks.get(k)
                if ts is not None and ti[k] in self._stale and ts.state in prefixes.LIVE_STATES:
                    return False
        return True

    def _remember_inputs(self, g, keys_):
        """What the engine holds of each uploaded task's _rootish and restrictions."""
        ro = g["rootish_override"]
        for i in np.flatnonzero(ro >= 0).tolist():
            self._rootish_h[keys_[i]] = int(ro[i])
        if "restr_flags" in g:
            rp, ri = g["restr_ptr"], g["restr_idx"]
            for i in np.flatnonzero(g["restr_flags"]):
                self._restr_h[keys_[i]] = (int(g["restr_flags"][i]), tuple(int(w) for w in ri[rp[i]:rp[i + 1]]))

    def _add_graph(self, new):
        """A later update_graph (scheduler.py:4662-4751) on the running engine; prefixes and
        groups map into the engine-wide tables. An independent graph whose tasks follow the
        earlier ones in priority (a new generation, :4713) runs its update_graph stimulus on
        the engine. A graph that depends on earlier tasks, carries restrictions, or whose
        user priority outranks earlier tasks (then every task's merged rank goes to the
        engine, dgp_set_priorities) is appended without placing, its tasks' valid workers
        go in, and its stimulus runs on the engine too (dgp_graph_stimulus); only when an
        earlier dependency is released / erred / forgotten (recomputed by the scheduler) is
        the stimulus the scheduler's own, the engine resynchronised after it (``_suspend``)."""
        s = self.scheduler
        g, keys_, prio_ = graph_from_tasks(new, [s.workers[a].nthreads if a in s.workers else 1 for a in self.workers],
                                    s.valid_workers, self.worker_index, earlier=self.task_index)
        restricted = "restr_flags" in g  # its stimulus the scheduler's, then the rows (dgp_update_restrictions)
        # a user priority that outranks earlier tasks (_set_priorities :4934-4981): the engine
        # takes every task's rank in the merged order (dgp_set_priorities) and the stimulus is
        # the scheduler's, then a resync
        outranks = prio_[0] <= self.max_priority
        if outranks and not hasattr(self.engine, "set_priorities"):
            raise NotImplementedError("a later graph whose tasks do not all follow the earlier ones in priority")
        if len(self.prefix_index) + sum(nm not in self.prefix_index for nm in g["prefix_names"]) > prefixes.PX:
            # more task prefixes over the session than the engine's table: the live ones and
            # this graph's in a compacted table (dgp_remap_prefixes + the dicts' resync)
            self._end_of_stimulus("the previous stimulus")
            if not self.active:
                return None
            self._compact_prefixes(list(g["prefix_names"]), resync=True)
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
            return None
        dependent = bool((g["dep_idx"] < 0).any())
        if restricted or outranks:
            self.engine.add_graph(g2, defer=True)
        else:
            self.engine.add_graph(g2)
        self.keys = self.keys + keys_
        self._note_prefixes(g)
        self.task_index.update(zip(keys_, range(n0, n0 + len(keys_))))
        self.prio_of = self.prio_of + prio_
        if outranks:  # every task's rank in the merged order (forgotten tasks keep theirs)
            order = sorted(range(len(self.prio_of)), key=self.prio_of.__getitem__)
            rank = np.empty(len(order), np.int64)
            rank[order] = np.arange(len(order))
            self.engine.set_priorities(rank)
            self.stats["reranked_graphs"] += 1
        g.pop("restr_flags", None)  # the rows go to the engine below (dgp_update_restrictions)
        self._remember_inputs(g, keys_)
        self.max_priority = max(self.max_priority, prio_[-1])
        self.stats["graphs"] += 1
        if dependent or restricted or outranks:
            if not outranks:
                self.stats["dependent_graphs" if dependent else "restricted_graphs"] += 1
            # the stimulus on the device (dgp_graph_stimulus), the new tasks' valid workers first
            if hasattr(self.engine, "graph_stimulus"):
                if restricted:
                    self._push_task_inputs(keys_)
                # released earlier dependencies are recomputed on the device when the engine
                # takes the scheduler's set orders (dgp_graph_stimulus_ordered)
                chain = loss.graph_cascade(new) if dependent else []
                ti = self.task_index
                order = None
                if chain and all(ts.key in ti and ts.prefix.name in self.prefix_index and ti[ts.key] not in self._stale
                                 for ts in chain):
                    order = loss.graph_orders(new, chain, lambda ts: ti[ts.key])
                    self.stats["graph_recomputes_on_device"] += 1
                stim = (self.engine.graph_stimulus(order) if order is not None else self.engine.graph_stimulus()) \
                    if self.active else None
                if stim is not None:
                    if order is not None:
                        self._recomputed = {ts.key for ts in chain}
                    self.stats["graph_stimuli_on_device"] += 1
                    self._fetch()
                    return keys_
            self._suspend("a later graph that depends on earlier tasks" if dependent else
                          "a later graph with restrictions" if restricted else "a later graph that outranks earlier tasks")
            for k in keys_:  # the new tasks, the earlier ones they wait on / add waiters to
                self._mark_dirty(k)
            return keys_
        self._fetch()
        return keys_

    def add_worker(self, scheduler=None, worker=None):
        """SchedulerPlugin.add_worker (diagnostics/plugin.py): Scheduler.add_worker calls it
        after check_idle_saturated(ws) and before bulk_schedule_unrunnable_after_adding_worker /
        stimulus_queue_slots_maybe_opened (scheduler.py:4398-4420). The engine adds the worker
        and makes the queue refill; the scheduler's own refill then consumes those decisions.
        The engine's worker index order is the scheduler's (SortedDict by address, :3746,
        :4353): the worker takes its address's place and every later index moves up by one on
        the device (dgp_add_worker_at); a worker that joins paused takes no refill."""
        self._enter()
        if not self.active or self.engine is None or worker in self.worker_index:
            return
        s = self.scheduler
        try:
            self._end_of_stimulus("the previous stimulus")
            if not self.active:
                return
            ws = s.workers[worker]
            running = ws.status.name == "running"
            # the engine's workers in address order (a removed one keeps its place, under a
            # name that sorts right after its address)
            pos = bisect.bisect_left(self.workers, worker)
            self.engine.add_worker(int(ws.nthreads), running=running, position=pos)
            self.workers.insert(pos, worker)
            if pos < len(self.workers) - 1:  # later workers moved up by one
                self.worker_index = {a: i for i, a in enumerate(self.workers) if not a.endswith(_REMOVED)}
                self._restr_h = {k: (fl, tuple(v + (v >= pos) for v in row)) for k, (fl, row) in self._restr_h.items()}
                self.stats["workers_inserted"] += 1
            else:
                self.worker_index[worker] = pos
            self._fetch()
            self.stats["workers_added"] += 1
            if not running:
                self.stats["workers_added_paused"] += 1
            self._window = (_ADD_WORKER_TRANSITIONS, None)
        except Exception as e:
            self.fallback(f"add_worker({worker}): {e}")

    def remove_worker(self, scheduler=None, worker=None, **kwargs):
        """SchedulerPlugin.remove_worker: Scheduler.remove_worker calls it after its own
        transitions (scheduler.py:5298-5302). The engine marks the worker removed
        (dgp_remove_worker: it leaves running / idle / saturated and total_nthreads and keeps
        its index, so the canonical order of the others stands). A worker that leaves with
        nothing processing and no last replica (retire_workers' drained worker: paused, its
        data copied elsewhere) runs no transition; its replicas went through the replica hook
        (dgp_remove_replicas) and the engine follows the removal on the device. Otherwise its
        processing tasks were released and re-placed and its lost results recomputed: by the
        engine (dgp_lose_worker, decided in ``_wrap_remove_worker`` before the scheduler's
        own code ran, whose transitions took those decisions), or, for a loss the engine does
        not restate, by the scheduler itself (the transition hook suspended the engine at the
        first of them) after which the engine takes the scheduler's state (dgp_sync_*)."""
        self._close_window()
        losing = self._losing
        token = getattr(self, "_loss_token", None)
        if token is not None and token[1] == worker:
            self._close_loss(token)  # the stimulus' transitions are over (:5298): close its window now
        if not self.active or self.engine is None or worker not in self.worker_index:
            return
        on_device = not self.suspended
        w = self.worker_index.pop(worker)
        self.removed.add(worker)
        self.workers[w] = worker + _REMOVED  # keeps its index and its place in address order
        if worker == losing and on_device:  # dgp_lose_worker decided the whole stimulus
            self._end_of_stimulus(f"remove_worker({worker})")
            return
        try:
            self.engine.remove_worker(w)
        except Exception as e:
            self.fallback(f"remove_worker({worker}): {e}")
            return
        if on_device:
            self.stats["workers_removed_on_device"] += 1
            self._fetch()  # none expected: a removal frees no slot
            self._end_of_stimulus(f"remove_worker({worker})")
            return
        self.stats["workers_removed"] += 1
        self._resync()

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
        self._window = None

    async def close(self):
        self.close_engine()

    # -------------------------------------------- other placement-input stimuli
    def _on_add_keys(self, kw):
        """add-keys (Scheduler.add_keys :7359-7391): new replicas of in-memory tasks reach
        the engine through the add_replica wrapper; nothing else changes."""

    def _on_long_running(self, kw):
        """long-running (Scheduler.handle_long_running :5817-5848): the task's prefix
        duration average takes the reported compute duration, the task leaves its worker's
        prefix counts (add_to_long_running :747-757) and frees a slot, then
        check_idle_saturated and the queue refill."""
        s = self.scheduler
        ts = s.tasks.get(kw.get("key"))
        if ts is None or ts.processing_on is None or ts.key not in self.task_index:
            return
        if ts in ts.processing_on.long_running:
            # a repeated report: the reference still averages the prefix duration, takes the
            # task out of the prefix counts again (add_to_long_running :747-757), then
            # check_idle_saturated and the queue refill (:5838-5848) -- not modelled on the
            # device: the scheduler decides this stimulus, then the engine takes its state
            self._suspend(f"long-running reported again for {ts.key!r}")
            self._mark_dirty(ts.key)
            return
        cd = kw.get("compute_duration")
        self._engine_op("long_running", self.task_index[ts.key], math.nan if cd is None else float(cd))

    def _on_worker_status_change(self, kw):
        """worker-status-change (Scheduler.handle_worker_status_change :5850-5883): a paused
        (or closing) worker leaves ``running``, idle, idle_task_count and saturated; one
        running again is checked (check_idle_saturated) and the queue refilled."""
        s = self.scheduler
        w = kw.get("worker")
        ws = s.workers.get(w) if isinstance(w, str) else w
        if ws is None:
            return
        st = kw.get("status")
        name = st if isinstance(st, str) else getattr(st, "name", str(st))
        if name == ws.status.name:
            return
        wi = self.worker_index.get(ws.address)
        if wi is None:
            self.fallback(f"worker-status-change of {ws.address}: not in the engine's table")
            return
        self._engine_op("set_worker_status", wi, 1 if name == "running" else 0)
        if self.active and name == "running":
            self._window = (_ADD_WORKER_TRANSITIONS, None)

    def _on_reschedule(self, kw):
        """reschedule (Scheduler._reschedule :7900-7924, the worker's Reschedule): a processing
        task released and placed again -- on the device (dgp_reschedule) when something needs
        it; otherwise (its release would release its dependencies) the scheduler decides and
        the engine resynchronises."""
        s = self.scheduler
        ts = s.tasks.get(kw.get("key"))
        if ts is None or ts.state != "processing":  # the reference returns without a transition
            return
        w = kw.get("worker")
        if w and ts.processing_on is not None and ts.processing_on.address != w:
            return
        if ts.key not in self.task_index:
            return
        if not (ts.waiters or ts.who_wants) or ts.has_lost_dependencies or ts.actor or \
                not hasattr(self.engine, "reschedule"):
            self._suspend(f"reschedule of {ts.key!r} is not restated by the engine")
            self._mark_dirty(ts.key)
            return
        if self._engine_op("reschedule", self.task_index[ts.key]) is None and self.active:
            self._suspend(f"reschedule of {ts.key!r}: {getattr(self.engine, 'refusal', 'refused by the engine')}")
            self._mark_dirty(ts.key)

    def _on_task_erred(self, kw):
        """task-erred (Scheduler.handle_task_erred :5799-5805 -> stimulus_task_erred
        :5094-5127, then the queue refill). A current run with no retries left errs: it leaves
        its worker (_exit_processing_common :3258), its waiting dependents err transitively,
        the dependencies nobody waits for any more are released (dgp_task_erred). A retry
        (:5116-5118: processing -> waiting through released) or a stale run's report from the
        worker it runs on (:5111-5113: processing -> released, re-waited when needed) of a task
        something needs is the reschedule's transitions (dgp_reschedule), then the refill
        (dgp_release_tasks of nothing); a task nobody needs: the scheduler's, then resync."""
        s = self.scheduler
        ts = s.tasks.get(kw.get("key"))
        if ts is None or ts.state != "processing" or ts.key not in self.task_index:
            return
        stale = ts.run_id != kw.get("run_id")
        if stale and not (ts.processing_on is not None and ts.processing_on.address == kw.get("worker")):
            return  # another worker's stale report: no transition (:5114)
        if not stale and ts.retries <= 0:
            self._engine_op("task_erred", self.task_index[ts.key])
            return
        what = "a stale run's task-erred" if stale else "a retry"
        if not (ts.waiters or ts.who_wants) or ts.has_lost_dependencies or ts.actor or \
                not hasattr(self.engine, "reschedule") or not hasattr(self.engine, "release_tasks"):
            self._suspend(f"{what} of {ts.key!r} is not restated by the engine")
            self._mark_dirty(ts.key)
            return
        if self._engine_op("reschedule", self.task_index[ts.key]) is None:
            if self.active:
                self._suspend(f"{what} of {ts.key!r}: {getattr(self.engine, 'refusal', 'refused by the engine')}")
                self._mark_dirty(ts.key)
            return
        try:  # stimulus_queue_slots_maybe_opened (:5805): after the transitions' placements
            self.engine.release_tasks(np.zeros(0, np.int32), np.zeros(0, np.uint8))
            self._fetch()
        except Exception as e:
            self.fallback(f"task-erred refill: {e}")
            return
        self.stats["erred_retries"] += 1

    def _on_client_desires_keys(self, kw):
        """client-desires-keys (:5398-5415): who_wants decides whether a finished task is
        released (_add_to_memory :3316, _transition_memory_released)."""
        s = self.scheduler
        t = [self.task_index[k] for k in kw.get("keys") or () if k in self.task_index
             and not (s.tasks.get(k) is not None and s.tasks[k].who_wants)]
        if t:
            self._engine_op("set_wanted", t, [1] * len(t))

    def _on_client_releases_keys(self, kw):
        """client-releases-keys (:5417-5430): tasks no longer wanted are released or
        forgotten -- results in memory, and cancelled work (waiting, processing, queued,
        no-worker). The engine follows on the device (dgp_release_tasks: the transitions in the
        scheduler's order from loss.release_plan, then the queue refill); a release the engine
        does not restate (a re-wait, an erred task, lost dependencies) is the scheduler's own
        stimulus, then a resync of those keys."""
        s = self.scheduler
        keys = [k for k in kw.get("keys") or () if k in self.task_index]
        if not keys:
            return
        plan = None
        if hasattr(self.engine, "release_tasks"):
            plan = loss.release_plan(s, kw.get("client"), keys)
        ti = self.task_index
        if plan is not None and all(ts.key in ti for ts, _ in plan):
            if not plan:
                return  # who_wants of another client only: nothing transitions
            if self._engine_op("release_tasks", [ti[ts.key] for ts, _ in plan], [1 if f else 0 for _, f in plan]) \
                    is not None or not self.active:
                return
        self._suspend("client-releases-keys")
        for k in keys:
            self._mark_dirty(k)

    def _on_update_data(self, kw):
        """update-data (:7394-7425): scattered data; a key of the engine's graph set to
        memory without a transition: the scheduler's stimulus, then a resync."""
        keys = [k for k in (kw.get("who_has") or {}) if k in self.task_index]
        if keys:
            self._suspend("update-data of tasks in the engine's graph")
            for k in keys:
                self._mark_dirty(k)

    def _on_heartbeat(self, kw, run):
        """heartbeat_worker (:4197-4252): the bandwidth EWMA (:4223-4226) and
        TaskPrefix.add_exec_time for the executing tasks (:4247-4252, :972-975) feed
        _calc_occupancy (:1884-1903) and worker_objective (:3131-3146)."""
        s = self.scheduler
        bw0 = s.bandwidth
        pref = {}
        for key in (kw.get("executing") or {}):
            ts = s.tasks.get(key)
            if ts is not None and ts.prefix.name in self.prefix_index:
                pref[ts.prefix.name] = ts.prefix
        before = {nm: (p.duration_average, p.max_exec_time) for nm, p in pref.items()}
        run()
        after = {nm: (p.duration_average, p.max_exec_time) for nm, p in pref.items()}
        if s.bandwidth == bw0 and before == after:
            return
        # each executing task's prefix in message order (add_exec_time is order-sensitive)
        ps, ds = [], []
        for key, dur in (kw.get("executing") or {}).items():
            ts = s.tasks.get(key)
            if ts is not None and ts.prefix.name in self.prefix_index:
                ps.append(self.prefix_index[ts.prefix.name])
                ds.append(float(dur))
        self._engine_op("heartbeat", float(s.bandwidth), ps, ds)

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
        ss = msg.get("startstops")
        if ss and len(ss) == 1 and ss[0].get("action") == "compute":  # the usual message
            a, b = float(ss[0]["start"]), float(ss[0]["stop"])
        else:
            a, b = _compute_interval(ss)
        return t, w, run, -1 if nbytes is None else int(nbytes), a, b

    async def handle_stream(self, comm, extra=None):
        """``Server.handle_stream`` (core.py:1015-1065) for the scheduler's worker streams,
        with one difference: the consecutive task-finished messages of one ``comm.read()``
        batch go to the engine in ONE call (``handle_task_finished_batch``). The handlers
        still run one message at a time, in arrival order, exactly as the reference loop
        calls them; a batch from a comm is one worker's (handle_worker's ``extra``)."""
        from distributed.comm.core import CommClosedError
        from distributed.utils import iscoroutinefunction

        extra = extra or {}
        s = self.scheduler
        try:
            while True:
                try:
                    msgs = await comm.read()
                except CommClosedError:
                    logger.info("Connection to %s has been closed.", comm.peer_address)
                    break
                if not isinstance(msgs, (tuple, list)):
                    msgs = (msgs,)
                closed = False
                run = []  # consecutive task-finished messages awaiting their engine call

                def flush():
                    if run:
                        self.handle_task_finished_batch([{**extra, **m} for m in run])
                        run.clear()

                for msg in msgs:
                    if msg == "OK":
                        break
                    op = msg.pop("op")
                    if not op:
                        logger.error("odd message %s", msg)
                        continue
                    if op == "close-stream":
                        closed = True
                        break
                    handler = s.stream_handlers[op]
                    if op == "task-finished" and handler == self.handle_task_finished:
                        run.append(msg)
                        continue
                    flush()
                    if iscoroutinefunction(handler):
                        await handler(**{**extra, **msg})
                    else:
                        handler(**{**extra, **msg})
                flush()
                if closed:
                    break
                await asyncio.sleep(0)
        finally:
            await comm.close()

    def handle_task_finished(self, key=None, worker=None, stimulus_id=None, **msg):
        """Stream handler "task-finished" (scheduler.py:3769 -> :5783-5797). The common case
        -- engine active, nothing left from the previous stimulus -- inline:
        ``handle_task_finished_batch`` of one message."""
        eng = self.engine
        post = getattr(eng, "tasks_finished_post", None)
        if (post is None or not self.active or not self.overlap or self.suspended or self.pending or self._msg_of
                or self._posted is not None):
            msg["key"], msg["worker"], msg["stimulus_id"] = key, worker, stimulus_id
            return self.handle_task_finished_batch((msg,))
        self._window = None
        s = self.scheduler
        try:
            post(*[(x,) for x in self._message_fields(key, worker, msg)])
        except Exception as e:
            self.fallback(f"tasks_finished: {e}")
        else:
            self._posted = self._posted_pairs = [(key, worker)]
        self._allowed.append(_STIMULUS_TRANSITIONS)
        try:
            type(s).handle_task_finished(s, key=key, worker=worker, stimulus_id=stimulus_id, **msg)
        finally:
            self._allowed.pop()
            self._settle()  # a message whose transitions asked for no decision
            self._expect_replicas.clear()
        if self.suspended:
            self._resync()
        if self.pending or self._msg_of:
            self._end_of_stimulus("task-finished")

    def handle_task_finished_batch(self, msgs):
        """Several task-finished messages in arrival order: ONE engine call (one PCIe copy),
        then the reference handler for each, consuming the engine's decisions in order. The
        call is posted (dgp_tasks_finished_post) and its answer taken at the first decision
        the handler's transitions ask for (``_settle``): the reference's Python up to there
        (stimulus_task_finished :5025-5090, _transition_processing_memory :2366-2420) runs
        while the device decides."""
        s = self.scheduler
        handler = type(s).handle_task_finished
        self._window = None  # _enter
        if self.suspended:
            self._resync()
        if self.pending or self._msg_of or self._posted is not None:
            self._end_of_stimulus("the previous stimulus")
        if self.active and self.engine is not None and msgs:
            if len(msgs) == 1:
                m = msgs[0]
                cols = [(x,) for x in self._message_fields(m["key"], m["worker"], m)]
            else:
                cols = list(zip(*[self._message_fields(m["key"], m["worker"], m) for m in msgs]))
            try:
                if self.overlap and hasattr(self.engine, "tasks_finished_post"):
                    self.engine.tasks_finished_post(*cols)
                    pairs = [(m["key"], m["worker"]) for m in msgs]
                    self._posted = pairs
                    self._posted_pairs = pairs if len(pairs) == 1 else set(pairs)
                else:
                    self._answer([(m["key"], m["worker"]) for m in msgs], *self.engine.tasks_finished(*cols))
            except Exception as e:
                self.fallback(f"tasks_finished: {e}")
        self._allowed.append(_STIMULUS_TRANSITIONS)
        try:
            for m in msgs:
                handler(s, **m)
        finally:
            self._allowed.pop()
            self._settle()  # a batch whose transitions asked for no decision
            self._expect_replicas.clear()
        if self.suspended:
            self._resync()
        if self.pending or self._msg_of:
            self._end_of_stimulus("task-finished")

    def _answer(self, pairs, status, n_new):
        status = status.tolist()
        # an already-in-memory report (add_keys) adds a replica after the placements of the
        # messages before it: those compute-task messages take who_has from the scheduler, as
        # built at their time (the reference's own _task_to_msg)
        if n_new:
            self._fetch(n_new, messages=len(status) == 1 or 2 not in status)
        self.stats["messages"] += len(pairs)
        expect, bad = self._expect_replicas, False
        for kw, st in zip(pairs, status):
            if st == 0:  # accepted: _add_to_memory adds this replica itself (:3296)
                expect.add(kw)
            elif st >= 3 and st != 4:
                bad = True
        # DGP_TF_RELEASE / _IMPOSSIBLE / _UNSUPPORTED: the reference reschedules or raises;
        # the engine does not follow those transitions
        if bad:
            self.fallback(f"task-finished answers {sorted(set(status))} the engine does not run")

    def _settle(self):
        """The posted batch's answer (dgp_tasks_finished_wait), then the replica additions
        the handler made before it, classified as add_replica would have at the time."""
        pairs = self._posted
        if pairs is None:
            return
        self._posted = None
        self._posted_pairs = ()
        try:
            self._answer(pairs, *self.engine.tasks_finished_wait())
        except Exception as e:
            self.fallback(f"tasks_finished: {e}")
        if not self._deferred_adds:
            return
        adds, self._deferred_adds = self._deferred_adds, []
        for ts, ws, had in adds:
            k = (ts.key, ws.address)
            if k in self._expect_replicas:
                self._expect_replicas.discard(k)
            elif not had:
                self._replica_event(ts, ws, +1)
