"""Drop-in WorkStealing whose balance() runs on the device.

``GPUWorkStealing`` subclasses the reference plugin (distributed/stealing.py:71-549) and
replaces only ``balance()`` (:401-503). Everything else stays the reference's own: the
stealable bins the ``transition`` hook keeps (:175-239), ``move_task_request`` /
``move_task_confirm`` (:279-399), the in-flight accounts, ``metrics``, the
``("request", log)`` event, ``story()`` and the ``steal-response`` stream handler, so
``extensions["stealing"]`` keeps its contract for the rest of the scheduler.

One balance() = one ``dgp_steal_balance`` call (PlacementEngine.steal_balance) on the
plugin's current state: workers (occupancy, processing, nbytes, idle / saturated), the
tasks of its bins with their levels, their dependencies and who_has, worker
restrictions (``valid_workers``), and the in-flight accounts of unconfirmed steals. The
device returns the ordered steal requests; they are applied here exactly as balance()
does: ``move_task_request`` per request, the log entry and both metrics, then
``check_idle_saturated(victim, occ=combined)`` for every victim the walk visited.

Order: within a bin the device takes tasks in ascending ``TaskState.priority`` and
victims in ascending worker address (the reference iterates Python sets, whose order
is hash-dependent; the golden fixtures pin the same canonical order).
"""
from __future__ import annotations

import math
from collections import Counter
from time import time

import numpy as np

try:  # the reference plugin (scheduler container); absent on the GPU box
    from distributed.stealing import WorkStealing, fast_tasks
except ImportError:  # pragma: no cover - exercised only where distributed is missing
    WorkStealing = object
    fast_tasks = set()


def steal_problem_from_state(plugin) -> tuple[dict, list, list]:
    """The dgp_steal_balance inputs of a WorkStealing plugin's scheduler state ->
    (problem dict, tasks in device order, workers in device order)."""
    s = plugin.scheduler
    wss = list(s.workers.values())
    widx = {ws.address: i for i, ws in enumerate(wss)}
    tasks = sorted(plugin.key_stealable, key=lambda ts: ts.priority)
    T, W = len(tasks), len(wss)
    data, didx, rows = [], {}, []
    for ts in tasks:
        r = []
        for dts in ts.dependencies:
            if dts not in didx:
                didx[dts] = len(data)
                data.append(dts)
            r.append(didx[dts])
        rows.append(sorted(r))
    dep_ptr = np.zeros(T + 1, np.int64)
    dep_ptr[1:] = np.cumsum([len(r) for r in rows])
    holders = [sorted(widx[ws.address] for ws in (dts.who_has or ())) for dts in data]
    hptr = np.zeros(len(data) + 1, np.int64)
    hptr[1:] = np.cumsum([len(h) for h in holders])
    p = dict(
        nthreads=np.array([ws.nthreads for ws in wss], np.int32),
        occ=np.array([ws.occupancy for ws in wss], np.float64),
        nproc=np.array([len(ws.processing) for ws in wss], np.int32),
        wnbytes=np.array([ws.nbytes for ws in wss], np.int64),
        idle=np.array([1 if ws.address in s.idle else 0 for ws in wss], np.uint8),
        sat=np.array([1 if ws in s.saturated else 0 for ws in wss], np.uint8),
        total_occ=float(s.total_occupancy), total_nthreads=int(s.total_nthreads), bandwidth=int(s.bandwidth),
        victim=np.array([widx[ts.processing_on.address] for ts in tasks], np.int32),
        # get_task_duration (scheduler.py:3024-3041), with its unknown_durations side effect
        duration=np.array([s.get_task_duration(ts) for ts in tasks], np.float64),
        fast=np.array([1 if ts.prefix.name in fast_tasks else 0 for ts in tasks], np.uint8),
        dep_ptr=dep_ptr, dep_idx=np.array([d for r in rows for d in r], np.int32),
        data_nbytes=np.array([dts.nbytes for dts in data], np.int64),
        data_get_nbytes=np.array([dts.get_nbytes() for dts in data], np.int64),
        holder_ptr=hptr, holder_idx=np.array([w for h in holders for w in h], np.int32),
        level_in=np.array([plugin.key_stealable[ts][1] for ts in tasks], np.int8),
        inflight_occ_in=np.array([float(plugin.in_flight_occupancy.get(ws, 0)) for ws in wss], np.float64),
        inflight_tasks_in=np.array([int(plugin.in_flight_tasks.get(ws, 0)) for ws in wss], np.int32),
    )
    flags = np.zeros(T, np.uint8)
    vrows = [[] for _ in range(T)]
    for i, ts in enumerate(tasks):
        if ts.worker_restrictions or ts.host_restrictions or ts.resource_restrictions:
            vw = s.valid_workers(ts)
            if vw is None:
                continue
            flags[i] = 1 | (2 if ts.loose_restrictions else 0)
            vrows[i] = sorted(widx[ws.address] for ws in vw)
    if flags.any():
        rp = np.zeros(T + 1, np.int64)
        rp[1:] = np.cumsum([len(r) for r in vrows])
        p.update(restr_ptr=rp, restr_idx=np.array([w for r in vrows for w in r], np.int32), restr_flags=flags)
    return p, tasks, wss


class GPUWorkStealing(WorkStealing):
    """WorkStealing with balance() on the MI355X (see the module docstring).

    ``engine_factory``: a callable returning the engine (default: PlacementEngine on
    ``device``); ``validate``: after applying, check that the plugin's in-flight accounts
    and the scheduler's idle / saturated sets equal the device's."""

    def __init__(self, scheduler, *, device: int = 0, engine_factory=None, validate: bool = False):
        self.device = device
        self.engine_factory = engine_factory
        self.validate = validate
        self.engine = None
        self.gpu_stats = Counter()
        super().__init__(scheduler)

    def _engine(self):
        if self.engine is None:
            if self.engine_factory is not None:
                self.engine = self.engine_factory()
            else:
                from .engine import PlacementEngine

                self.engine = PlacementEngine(self.device)
        return self.engine

    def balance(self) -> None:
        s = self.scheduler
        start = time()
        # the early exits of balance() (stealing.py:409-411): no thief, or every worker one
        if not s.idle or len(s.idle) == len(s.workers):
            return
        p, tasks, wss = steal_problem_from_state(self)
        out = self._engine().steal_balance(p)
        log = []
        for k in range(len(out["st_task"])):
            ts = tasks[int(out["st_task"][k])]
            victim, thief = wss[int(out["st_victim"][k])], wss[int(out["st_thief"][k])]
            level = int(out["st_level"][k])
            cost = float(out["st_cost"][k])
            self.move_task_request(ts, victim, thief)  # :466
            log.append((start, level, ts.key, cost, victim.address, float(out["st_occ_victim"][k]), thief.address,
                        float(out["st_occ_thief"][k])))
            self.metrics["request_count_total"][level] += 1  # :479-480
            self.metrics["request_cost_total"][level] += cost
        for i in np.flatnonzero(out["checked"]):  # check_idle_saturated(victim, occ=combined) :498-500
            ws = wss[int(i)]
            s.check_idle_saturated(ws, occ=self._combined_occupancy(ws))
        self.gpu_stats["balance_calls"] += 1
        self.gpu_stats["steal_requests"] += len(log)
        if self.validate:
            self._validate(out, wss)
        if log:
            self.log(("request", log))
            self.count += 1
        stop = time()
        if s.digests:
            s.digests["steal-duration"].add(stop - start)

    def _validate(self, out, wss):
        s = self.scheduler
        for i, ws in enumerate(wss):
            io = float(self.in_flight_occupancy.get(ws, 0))
            if not (io == out["inflight_occ"][i] or (math.isnan(io) and math.isnan(out["inflight_occ"][i]))):
                raise AssertionError(f"gpu-stealing: in-flight occupancy of {ws.address}: {io} != {out['inflight_occ'][i]}")
            if int(self.in_flight_tasks.get(ws, 0)) != int(out["inflight_tasks"][i]):
                raise AssertionError(f"gpu-stealing: in-flight tasks of {ws.address}")
            if (ws.address in s.idle) != bool(out["idle_after"][i]) or (ws in s.saturated) != bool(out["sat_after"][i]):
                raise AssertionError(f"gpu-stealing: idle / saturated of {ws.address}")
