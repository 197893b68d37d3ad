"""Drop-in WorkStealing whose balance() runs on the device.

``GPUWorkStealing`` subclasses the reference plugin (distributed/stealing.py:71-549) and
replaces only ``balance()`` (:401-503). Everything else stays the reference's own: the
stealable bins the ``transition`` hook keeps (:175-239), ``move_task_request`` /
``move_task_confirm`` (:279-399), the in-flight accounts, ``metrics``, the
``("request", log)`` event, ``story()`` and the ``steal-response`` stream handler, so
``extensions["stealing"]`` keeps its contract for the rest of the scheduler.

One balance() = one ``dgp_steal_balance`` call (PlacementEngine.steal_balance) on the
plugin's current state (the task rows kept incrementally, ``StealRows``): workers
(occupancy, processing, nbytes, idle / saturated), the
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
    p = _worker_columns(plugin, s, wss)
    p.update(
        victim=np.array([widx[ts.processing_on.address] for ts in tasks], np.int32),
        # get_task_duration (scheduler.py:3024-3041), with its unknown_durations side effect
        duration=np.array([s.get_task_duration(ts) for ts in tasks], np.float64),
        fast=np.array([1 if ts.prefix.name in fast_tasks else 0 for ts in tasks], np.uint8),
        dep_ptr=dep_ptr, dep_idx=np.array([d for r in rows for d in r], np.int32),
        data_nbytes=np.array([dts.nbytes for dts in data], np.int64),
        data_get_nbytes=np.array([dts.get_nbytes() for dts in data], np.int64),
        holder_ptr=hptr, holder_idx=np.array([w for h in holders for w in h], np.int32),
        level_in=np.array([plugin.key_stealable[ts][1] for ts in tasks], np.int8),
    )
    _restriction_rows(p, s, tasks, widx)
    return p, tasks, wss


class StealRows:
    """The task rows of the steal problem, kept as the plugin's transition hook fills and
    empties its bins (``put_key_in_stealable`` / ``remove_key_from_stealable``,
    stealing.py:218-239), so one ``balance()`` gathers them instead of rebuilding them: per
    task (one numpy row slot) its bin worker, level, fast flag, prefix and dependency ids
    (ascending, into a refcounted table of the dependency TaskStates), ordered by
    (priority, arrival). Read at balance time, as the full rebuild does: durations (per
    prefix), restrictions and the dependencies' nbytes / holders (one pass over the
    distinct dependencies)."""

    KD = 4  # dependency ids held in the slot row; longer rows keep the rest in ``more``

    def __init__(self):
        from sortedcontainers import SortedList

        self.slot = {}  # TaskState -> row slot
        self.task, self.key, self.free = [], [], []
        self.order = SortedList()  # (priority, arrival, slot): ties in arrival order
        self.arrival = 0
        cap = 1024
        self.lvl = np.zeros(cap, np.int8)
        self.fst = np.zeros(cap, np.uint8)
        self.pfx = np.zeros(cap, np.int32)
        self.vic = np.zeros(cap, np.int32)
        self.nd = np.zeros(cap, np.int32)
        self.dmat = np.zeros((cap, self.KD), np.int64)
        self.more = {}  # slot -> dependency ids beyond the first KD
        self.data_id, self.data, self.data_ref, self.data_free = {}, [], [], []
        self.prefix_id, self.prefixes = {}, []  # TaskPrefix name -> code, code -> TaskPrefix
        self.addr_id, self.addrs = {}, []  # worker address -> code

    def __len__(self):
        return len(self.slot)

    def _grow(self):
        cap = 2 * len(self.lvl)
        for nm in ("lvl", "fst", "pfx", "vic", "nd"):
            a = getattr(self, nm)
            b = np.zeros(cap, a.dtype)
            b[:len(a)] = a
            setattr(self, nm, b)
        d = np.zeros((cap, self.KD), np.int64)
        d[:len(self.dmat)] = self.dmat
        self.dmat = d

    def _code(self, table, items, key, obj):
        c = table.get(key)
        if c is None:
            c = table[key] = len(items)
            items.append(obj)
        return c

    def put(self, ts, worker: str, level: int) -> None:
        if ts in self.slot:
            self.remove(ts)
        ids = []
        for dts in ts.dependencies:
            j = self.data_id.get(dts)
            if j is None:
                if self.data_free:
                    j = self.data_free.pop()
                    self.data[j] = dts
                    self.data_ref[j] = 0
                else:
                    j = len(self.data)
                    self.data.append(dts)
                    self.data_ref.append(0)
                self.data_id[dts] = j
            self.data_ref[j] += 1
            ids.append(j)
        ids.sort()
        if self.free:
            i = self.free.pop()
        else:
            i = len(self.task)
            self.task.append(None)
            self.key.append(None)
            if i >= len(self.lvl):
                self._grow()
        key = (ts.priority, self.arrival, i)
        self.arrival += 1
        self.task[i], self.key[i] = ts, key
        self.lvl[i] = level
        pf = ts.prefix
        self.fst[i] = 1 if pf.name in fast_tasks else 0
        self.pfx[i] = self._code(self.prefix_id, self.prefixes, pf.name, pf)
        self.vic[i] = self._code(self.addr_id, self.addrs, worker, worker)
        self.nd[i] = len(ids)
        k = min(len(ids), self.KD)
        self.dmat[i, :k] = ids[:k]
        if len(ids) > self.KD:
            self.more[i] = ids[self.KD:]
        self.slot[ts] = i
        self.order.add(key)

    def remove(self, ts) -> None:
        i = self.slot.pop(ts, None)
        if i is None:
            return
        self.order.remove(self.key[i])
        n = int(self.nd[i])
        for j in self.dmat[i, :min(n, self.KD)].tolist() + self.more.pop(i, []):
            self.data_ref[j] -= 1
            if self.data_ref[j] == 0:
                del self.data_id[self.data[j]]
                self.data[j] = None
                self.data_free.append(j)
        self.task[i] = self.key[i] = None
        self.free.append(i)

    def clear(self) -> None:
        self.__init__()

    def problem(self, plugin) -> tuple[dict, list, list]:
        """Same result as ``steal_problem_from_state(plugin)`` (up to the numbering of the
        dependencies, which the device does not order by)."""
        s = plugin.scheduler
        wss = list(s.workers.values())
        widx = {ws.address: i for i, ws in enumerate(wss)}
        T = len(self.order)
        rows = np.fromiter((k[2] for k in self.order), np.int64, T)
        tasks = [self.task[i] for i in rows.tolist()]
        p = _worker_columns(plugin, s, wss)
        amap = np.array([widx.get(a, -1) for a in self.addrs] or [0], np.int32)
        p["victim"] = amap[self.vic[rows]]
        # get_task_duration (scheduler.py:3024-3041) per prefix; its unknown_durations side
        # effect for the tasks of prefixes without a duration
        pd = np.array([pf.duration_average for pf in self.prefixes] or [0.0], np.float64)
        dur = pd[self.pfx[rows]]
        for k in np.flatnonzero(~(dur >= 0)).tolist():
            dur[k] = s.get_task_duration(tasks[k])
        p["duration"] = dur
        p["fast"] = self.fst[rows]
        p["level_in"] = self.lvl[rows]
        cnt = self.nd[rows].astype(np.int64)
        dep_ptr = np.zeros(T + 1, np.int64)
        np.cumsum(cnt, out=dep_ptr[1:])
        gids = np.empty(int(dep_ptr[-1]), np.int64)
        r_, j_ = np.nonzero(np.arange(self.KD)[None, :] < np.minimum(cnt, self.KD)[:, None])
        gids[dep_ptr[r_] + j_] = self.dmat[rows[r_], j_]
        for r in np.flatnonzero(cnt > self.KD).tolist():
            ex = self.more[int(rows[r])]
            gids[dep_ptr[r] + self.KD:dep_ptr[r + 1]] = ex
        uniq, inv = np.unique(gids, return_inverse=True)  # monotone: rows stay ascending
        data = [self.data[j] for j in uniq.tolist()]
        holders = [sorted(widx[ws.address] for ws in (dts.who_has or ())) for dts in data]
        hptr = np.zeros(len(data) + 1, np.int64)
        np.cumsum([len(h) for h in holders], out=hptr[1:])
        p.update(dep_ptr=dep_ptr, dep_idx=inv.astype(np.int32).reshape(-1),
                 data_nbytes=np.array([dts.nbytes for dts in data], np.int64),
                 data_get_nbytes=np.array([dts.get_nbytes() for dts in data], np.int64),
                 holder_ptr=hptr, holder_idx=np.array([w for h in holders for w in h], np.int32))
        _restriction_rows(p, s, tasks, widx)
        return p, tasks, wss


def _worker_columns(plugin, s, wss) -> dict:
    return dict(
        nthreads=np.array([ws.nthreads for ws in wss], np.int32),
        occ=np.array([ws.occupancy for ws in wss], np.float64),
        nproc=np.array([len(ws.processing) for ws in wss], np.int32),
        wnbytes=np.array([ws.nbytes for ws in wss], np.int64),
        idle=np.array([1 if ws.address in s.idle else 0 for ws in wss], np.uint8),
        sat=np.array([1 if ws in s.saturated else 0 for ws in wss], np.uint8),
        total_occ=float(s.total_occupancy), total_nthreads=int(s.total_nthreads), bandwidth=int(s.bandwidth),
        inflight_occ_in=np.array([float(plugin.in_flight_occupancy.get(ws, 0)) for ws in wss], np.float64),
        inflight_tasks_in=np.array([int(plugin.in_flight_tasks.get(ws, 0)) for ws in wss], np.int32),
    )


def _restriction_rows(p, s, tasks, widx) -> None:
    """valid_workers (scheduler.py:3043-3107) of the restricted tasks, read at balance time."""
    T = len(tasks)
    flags = np.zeros(T, np.uint8)
    vrows = {}
    for i, ts in enumerate(tasks):
        if ts.worker_restrictions or ts.host_restrictions or ts.resource_restrictions:
            vw = s.valid_workers(ts)
            if vw is None:
                continue
            flags[i] = 1 | (2 if ts.loose_restrictions else 0)
            vrows[i] = sorted(widx[ws.address] for ws in vw)
    if vrows:
        rp = np.zeros(T + 1, np.int64)
        for i, r in vrows.items():
            rp[i + 1] = len(r)
        np.cumsum(rp, out=rp)
        p.update(restr_ptr=rp, restr_idx=np.array([w for i in sorted(vrows) for w in vrows[i]], np.int32),
                 restr_flags=flags)


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
        self.rows = StealRows()  # before the reference __init__: its hooks may fill the bins
        super().__init__(scheduler)

    # the bins' task rows follow the reference hooks (stealing.py:218-239, :511-516)
    def put_key_in_stealable(self, ts) -> None:
        super().put_key_in_stealable(ts)
        r = self.key_stealable.get(ts)
        if r is not None:
            self.rows.put(ts, r[0], r[1])

    def remove_key_from_stealable(self, ts) -> None:
        super().remove_key_from_stealable(ts)
        self.rows.remove(ts)

    def restart(self, scheduler) -> None:
        super().restart(scheduler)
        self.rows.clear()

    def problem(self):
        """The dgp_steal_balance inputs of the current state (the incremental rows; rebuilt
        from the bins if anything changed them outside the hooks)."""
        if len(self.rows) != len(self.key_stealable):
            self.gpu_stats["rows_rebuilt"] += 1
            self.rows.clear()
            for ts, (worker, level) in self.key_stealable.items():
                self.rows.put(ts, worker, level)
        return self.rows.problem(self)

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
        p, tasks, wss = self.problem()
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
