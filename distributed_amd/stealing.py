"""Drop-in WorkStealing whose balance() runs on the device.

``GPUWorkStealing`` subclasses the reference plugin (distributed/stealing.py:71-549) and
replaces only ``balance()`` (:401-503). Everything else stays the reference's own: the
stealable bins the ``transition`` hook keeps (:175-239), ``move_task_request`` /
``move_task_confirm`` (:279-399), the in-flight accounts, ``metrics``, the
``("request", log)`` event, ``story()`` and the ``steal-response`` stream handler, so
``extensions["stealing"]`` keeps its contract for the rest of the scheduler.

One balance() = one ``dgp_steal_balance`` call (PlacementEngine.steal_balance) on the
plugin's current state (the task rows and their dependencies' who_has kept incrementally,
``StealRows``; ``balance_plan``): workers
(occupancy, processing, nbytes, idle / saturated), the
tasks of its bins with their levels, their dependencies and who_has, worker
restrictions (``valid_workers``), and the in-flight accounts of unconfirmed steals. The
device returns the ordered steal requests; they are applied here exactly as balance()
does: ``move_task_request`` per request, the log entry and both metrics, then
``check_idle_saturated(victim, occ=combined)`` for every victim the walk visited.

Order: within a bin the device takes tasks in ascending ``TaskState.priority`` (then
arrival in the bin; the rows go unsorted, the device sorts them: dgp_steal_order) and
victims in ascending worker address (the reference iterates Python sets, whose order
is hash-dependent; the golden fixtures pin the same canonical order).
"""
from __future__ import annotations

import gc
import itertools
import math
import operator
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
    _restriction_rows(p, s, list(enumerate(tasks)), T, widx)
    return p, tasks, wss


def pack_priority(pr):
    """``TaskState.priority`` = (-user priority, generation, dask.order position)
    (scheduler.py:4719-4724) as one int64 of the same order, or None when it does not fit
    (then the host orders the rows)."""
    try:
        a, b, c = pr
    except (TypeError, ValueError):
        return None
    if type(a) is int and type(b) is int and type(c) is int and -(1 << 15) <= a < (1 << 15) and 0 <= b < (1 << 20) \
            and 0 <= c < (1 << 27):
        return ((a + (1 << 15)) << 47) | (b << 27) | c
    return None


class StealRows:
    """The steal problem's rows, kept as the plugin's hooks change its state, so that one
    ``balance()`` gathers them with numpy instead of visiting TaskStates:

    * task rows (one slot each, filled and emptied by ``put_key_in_stealable`` /
      ``remove_key_from_stealable``, stealing.py:218-239): bin worker, level, fast flag,
      prefix, dependency ids (into the dependency table), the packed priority and arrival
      (the device orders the rows by them, dgp_steal_order), a restrictions flag;
    * the dependency table (refcounted by the task rows): nbytes, get_nbytes() and who_has
      as worker-address codes, kept by the scheduler's replica hooks (add_replica /
      remove_replica / remove_all_replicas, scheduler.py:3148-3171, wrapped by the plugin).

    Read at balance time: worker columns, durations (per prefix), restrictions (restricted
    rows only)."""

    KD = 4  # dependency ids held in the slot row; longer rows keep the rest in ``more``
    HM = 8  # holders held in the dependency row; more in ``hmore``

    def __init__(self):
        self.slot = {}  # TaskState -> row slot
        self.task, self.free = [], []
        self.arrival = 0
        cap = 1024
        self.live = np.zeros(cap, bool)
        self.lvl = np.zeros(cap, np.int8)
        self.fst = np.zeros(cap, np.uint8)
        self.pfx = np.zeros(cap, np.int32)
        self.vic = np.zeros(cap, np.int32)
        self.nd = np.zeros(cap, np.int32)
        self.dmat = np.zeros((cap, self.KD), np.int64)
        self.pk = np.zeros(cap, np.int64)
        self.arr = np.zeros(cap, np.int64)
        self.rst = np.zeros(cap, np.uint8)
        self.more = {}  # slot -> dependency ids beyond the first KD
        self.pk_bad = {}  # slot -> a priority pack_priority cannot hold
        self.data_id, self.data, self.data_free = {}, [], []
        dcap = 1024
        self.data_ref = np.zeros(dcap, np.int64)  # task rows referencing each dependency
        self.dnb = np.zeros(dcap, np.int64)
        self.dgnb = np.zeros(dcap, np.int64)
        self.hold = np.zeros((dcap, self.HM), np.int32)
        self.hcnt = np.zeros(dcap, np.int32)
        self.hmore = {}  # data slot -> holder codes beyond HM
        self.prefix_id, self.prefixes = {}, []  # TaskPrefix name -> code, code -> TaskPrefix
        self.addr_id, self.addrs = {}, []  # worker address -> code

    def __len__(self):
        return len(self.slot)

    @staticmethod
    def _grown(a, cap):
        b = np.zeros((cap,) + a.shape[1:], a.dtype)
        b[:len(a)] = a
        return b

    def _grow(self):
        cap = 2 * len(self.lvl)
        for nm in ("live", "lvl", "fst", "pfx", "vic", "nd", "dmat", "pk", "arr", "rst"):
            setattr(self, nm, self._grown(getattr(self, nm), cap))

    def _code(self, table, items, key, obj):
        c = table.get(key)
        if c is None:
            c = table[key] = len(items)
            items.append(obj)
        return c

    # ------------------------------------------------------------- dependency table
    def _new_data(self, dts):
        if self.data_free:
            j = self.data_free.pop()
            self.data[j] = dts
            self.data_ref[j] = 0
        else:
            j = len(self.data)
            self.data.append(dts)
            if j >= len(self.dnb):
                cap = 2 * len(self.dnb)
                for nm in ("data_ref", "dnb", "dgnb", "hold", "hcnt"):
                    setattr(self, nm, self._grown(getattr(self, nm), cap))
            self.data_ref[j] = 0
        self.data_id[dts] = j
        self.dnb[j] = dts.nbytes
        self.dgnb[j] = dts.get_nbytes()
        self.hcnt[j] = 0
        self.hmore.pop(j, None)
        for ws in dts.who_has or ():
            self._hold_add(j, self._code(self.addr_id, self.addrs, ws.address, ws.address))
        return j

    def _hold_add(self, j, c):
        n = int(self.hcnt[j])
        if c in self.hold[j, :min(n, self.HM)] or c in self.hmore.get(j, ()):
            return
        if n < self.HM:
            self.hold[j, n] = c
        else:
            self.hmore.setdefault(j, []).append(c)
        self.hcnt[j] = n + 1

    def _hold_remove(self, j, c):
        n = int(self.hcnt[j])
        ex = self.hmore.get(j)
        row = self.hold[j]
        for q in range(min(n, self.HM)):
            if row[q] == c:  # the last holder takes its place
                if ex:
                    row[q] = ex.pop()
                    if not ex:
                        del self.hmore[j]
                else:
                    row[q] = row[n - 1]
                self.hcnt[j] = n - 1
                return
        if ex and c in ex:
            ex.remove(c)
            if not ex:
                del self.hmore[j]
            self.hcnt[j] = n - 1

    def replica(self, ts, address, sign):
        """SchedulerState.add_replica / remove_replica of (ts, worker) (the plugin's hooks)."""
        j = self.data_id.get(ts)
        if j is None:
            return
        c = self._code(self.addr_id, self.addrs, address, address)
        if sign > 0:
            self.dnb[j] = ts.nbytes
            self.dgnb[j] = ts.get_nbytes()
            self._hold_add(j, c)
        else:
            self._hold_remove(j, c)

    def replicas_cleared(self, ts):
        """SchedulerState.remove_all_replicas(ts)."""
        j = self.data_id.get(ts)
        if j is not None:
            self.hcnt[j] = 0
            self.hmore.pop(j, None)

    # ------------------------------------------------------------------ task rows
    def put(self, ts, worker: str, level: int) -> None:
        if ts in self.slot:
            self.remove(ts)
        ids = []
        for dts in ts.dependencies:
            j = self.data_id.get(dts)
            if j is None:
                j = self._new_data(dts)
            self.data_ref[j] += 1
            ids.append(j)
        ids.sort()
        if self.free:
            i = self.free.pop()
        else:
            i = len(self.task)
            self.task.append(None)
            if i >= len(self.lvl):
                self._grow()
        self.task[i] = ts
        self.live[i] = True
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
        pk = pack_priority(ts.priority)
        if pk is None:
            self.pk_bad[i] = ts.priority
            pk = 0
        self.pk[i] = pk
        self.arr[i] = self.arrival
        self.arrival += 1
        self.rst[i] = 1 if (ts.worker_restrictions or ts.host_restrictions or ts.resource_restrictions) else 0
        self.slot[ts] = i

    def remove(self, ts) -> None:
        i = self.slot.pop(ts, None)
        if i is None:
            return
        n = int(self.nd[i])
        for j in self.dmat[i, :min(n, self.KD)].tolist() + self.more.pop(i, []):
            self.data_ref[j] -= 1
            if self.data_ref[j] == 0:
                del self.data_id[self.data[j]]
                self.data[j] = None
                self.hcnt[j] = 0
                self.hmore.pop(j, None)
                self.data_free.append(j)
        self.pk_bad.pop(i, None)
        self.live[i] = False
        self.task[i] = None
        self.free.append(i)

    def remove_many(self, tss, slots) -> None:
        """``remove`` of many rows at once (the requested tasks of one balance()): ``slots``
        their row slots, in the order of ``tss``."""
        slots = np.asarray(slots, np.int64)
        if not len(slots):
            return
        pop = self.slot.pop
        for ts in tss:
            pop(ts, None)
        n = self.nd[slots].astype(np.int64)
        inrow = np.arange(self.KD)[None, :] < np.minimum(n, self.KD)[:, None]
        ids = [self.dmat[slots][inrow]]
        if self.more:
            more = self.more
            ids += [np.asarray(more.pop(i), np.int64) for i in slots[n > self.KD].tolist() if i in more]
        ids = np.concatenate(ids)
        dec = np.bincount(ids, minlength=len(self.data))
        touched = np.flatnonzero(dec)
        self.data_ref[touched] -= dec[touched]
        for j in touched[self.data_ref[touched] == 0].tolist():
            del self.data_id[self.data[j]]
            self.data[j] = None
            self.hmore.pop(j, None)
            self.data_free.append(j)
        gone = touched[self.data_ref[touched] == 0]
        self.hcnt[gone] = 0
        if self.pk_bad:
            for i in slots.tolist():
                self.pk_bad.pop(i, None)
        self.live[slots] = False
        task = self.task
        sl = slots.tolist()
        for i in sl:
            task[i] = None
        self.free.extend(sl)

    def clear(self) -> None:
        self.__init__()

    def problem(self, plugin) -> tuple[dict, np.ndarray, list]:
        """The dgp_steal_balance inputs of the current state -> (problem dict, the row slot
        of each problem task, workers in device order). The rows go in slot order with
        their (priority, arrival) keys; the device orders them (dgp_steal_order)."""
        s = plugin.scheduler
        wss = list(s.workers.values())
        widx = {ws.address: i for i, ws in enumerate(wss)}
        n = len(self.task)
        rows = np.flatnonzero(self.live[:n])
        T = len(rows)
        sel = slice(0, n) if T == n else rows  # no free slot: the columns are read as views
        p = _worker_columns(plugin, s, wss)
        amap = np.array([widx.get(a, -1) for a in self.addrs] or [0], np.int32)
        p["victim"] = amap[self.vic[sel]]
        # get_task_duration (scheduler.py:3024-3041) per prefix; its unknown_durations side
        # effect for the tasks of prefixes without a duration
        pd = np.array([pf.duration_average for pf in self.prefixes] or [0.0], np.float64)
        dur = pd[self.pfx[sel]]
        for k in np.flatnonzero(~(dur >= 0)).tolist():
            dur[k] = s.get_task_duration(self.task[int(rows[k])])
        p["duration"] = dur
        p["fast"] = self.fst[sel]
        p["level_in"] = self.lvl[sel]
        cnt = self.nd[sel].astype(np.int64)
        dep_ptr = np.zeros(T + 1, np.int64)
        np.cumsum(cnt, out=dep_ptr[1:])
        inrow = np.arange(self.KD)[None, :] < np.minimum(cnt, self.KD)[:, None]
        if not self.more:  # every row in its slot: the row-major selection is the CSR
            gids = self.dmat[sel][inrow]
        else:
            gids = np.empty(int(dep_ptr[-1]), np.int64)
            r_, j_ = np.nonzero(inrow)
            gids[dep_ptr[r_] + j_] = self.dmat[rows[r_], j_]
            for r in np.flatnonzero(cnt > self.KD).tolist():
                gids[dep_ptr[r] + self.KD:dep_ptr[r + 1]] = self.more[int(rows[r])]
        nd_ = len(self.data)
        hc = self.hcnt[:nd_].astype(np.int64)
        hptr = np.zeros(nd_ + 1, np.int64)
        np.cumsum(hc, out=hptr[1:])
        inline = np.minimum(hc, self.HM)
        m = np.arange(self.HM)[None, :] < inline[:, None]
        hm = np.where(m, amap[self.hold[:nd_]], np.iinfo(np.int32).max)
        if self.hmore:  # rows with more holders than HM: their full lists
            hidx = np.empty(int(hptr[-1]), np.int32)
            big = np.zeros(nd_, bool)
            big[list(self.hmore)] = True
            mm = m & ~big[:, None]
            hm_small = np.sort(np.where(mm, hm, np.iinfo(np.int32).max), axis=1)
            rr, cc = np.nonzero(np.arange(self.HM)[None, :] < np.where(big, 0, inline)[:, None])
            hidx[hptr[rr] + cc] = hm_small[rr, cc]
            for j, ex in self.hmore.items():
                hidx[hptr[j]:hptr[j + 1]] = np.sort(np.concatenate([hm[j, :self.HM], amap[np.asarray(ex, np.int64)]]))
        else:
            multi = np.flatnonzero(inline > 1)  # most data have one holder: sort only the others
            if len(multi):
                hm[multi] = np.sort(hm[multi], axis=1)
            hidx = hm[m]
        p.update(dep_ptr=dep_ptr, dep_idx=gids.astype(np.int32), data_nbytes=self.dnb[:nd_],
                 data_get_nbytes=self.dgnb[:nd_], holder_ptr=hptr, holder_idx=hidx.astype(np.int32))
        if self.pk_bad:  # priorities that do not pack: the rows' ranks in the host's order
            keys = [(self.pk_bad[i] if i in self.pk_bad else self.task[i].priority, int(self.arr[i]))
                    for i in rows.tolist()]
            order = sorted(range(T), key=keys.__getitem__)
            rank = np.empty(T, np.int64)
            rank[order] = np.arange(T)
            p["task_prio"], p["task_arrival"] = rank, np.zeros(T, np.int64)
        else:
            p["task_prio"], p["task_arrival"] = self.pk[sel], self.arr[sel]
        rpos = np.flatnonzero(self.rst[sel]).tolist()
        if rpos:
            _restriction_rows(p, s, [(k, self.task[int(rows[k])]) for k in rpos], T, widx)
        return p, rows, wss


def ordered_problem(p, slots):
    """A StealRows problem (rows in slot order with their task_prio / task_arrival keys) with
    its tasks put in the device's walk order (ascending priority, then arrival) -- the
    layout of steal_problem_from_state; for tests and checks. Returns (problem, slots)."""
    perm = np.lexsort((p["task_arrival"], p["task_prio"]))
    q = {k: v for k, v in p.items() if k not in ("task_prio", "task_arrival")}
    for k in ("victim", "duration", "fast", "level_in"):
        q[k] = p[k][perm]
    cnt = np.diff(p["dep_ptr"])[perm]
    dp = np.zeros(len(perm) + 1, np.int64)
    np.cumsum(cnt, out=dp[1:])
    q["dep_ptr"] = dp
    q["dep_idx"] = np.concatenate([p["dep_idx"][p["dep_ptr"][t]:p["dep_ptr"][t + 1]] for t in perm] or
                                  [np.zeros(0, np.int32)]).astype(np.int32)
    if p.get("restr_flags") is not None:
        rc = np.diff(p["restr_ptr"])[perm]
        rp = np.zeros(len(perm) + 1, np.int64)
        np.cumsum(rc, out=rp[1:])
        q["restr_ptr"] = rp
        q["restr_idx"] = np.concatenate([p["restr_idx"][p["restr_ptr"][t]:p["restr_ptr"][t + 1]] for t in perm] or
                                        [np.zeros(0, np.int32)]).astype(np.int32)
        q["restr_flags"] = p["restr_flags"][perm]
    return q, np.asarray(slots)[perm]


def thief_comm_bytes(p, prow, thief) -> np.ndarray:
    """Per request: the bytes of its task's dependencies the thief does not hold --
    ``get_comm_cost(ts, thief)``'s sum (scheduler.py:3006-3022, raw ``nbytes``) -- from the
    problem arrays (``prow``: each request's problem row, ``thief``: its thief's index)."""
    dp, di = p["dep_ptr"], p["dep_idx"]
    a, b = dp[prow], dp[prow + 1]
    cnt = (b - a).astype(np.int64)
    K = len(prow)
    if not K or not cnt.sum():
        return np.zeros(K, np.int64)
    k_of = np.repeat(np.arange(K), cnt)  # one entry per (request, dependency)
    first = np.cumsum(cnt) - cnt
    d = di[np.repeat(a, cnt) + (np.arange(len(k_of)) - np.repeat(first, cnt))].astype(np.int64)
    hp, hi = p["holder_ptr"], p["holder_idx"]
    hn = (hp[d + 1] - hp[d]).astype(np.int64)
    e_of = np.repeat(np.arange(len(d)), hn)  # one entry per (dependency entry, holder)
    hfirst = np.cumsum(hn) - hn
    h = hi[np.repeat(hp[d], hn) + (np.arange(len(e_of)) - np.repeat(hfirst, hn))]
    held = np.zeros(len(d), bool)
    held[e_of[h == thief[k_of[e_of]]]] = True
    nb = np.where(held, 0, p["data_nbytes"][d]).astype(np.int64)
    out = np.zeros(K, np.int64)
    np.add.at(out, k_of, nb)
    return out


def apply_requests(plugin, out, p, rows, wss, start) -> list:
    """The requests of one balance(), applied in bulk -- what ``move_task_request`` does per
    request (stealing.py:279-321: the task leaves its bin, a ``steal-request`` message to the
    victim, the in-flight record and accounts, ``_add_to_in_flight`` :191-199), the log entry
    and both metrics (:466-480) -- with the same results. The in-flight accounts are the
    device's (its walk carried them in the reference's operation order: ``inflight_occ`` /
    ``inflight_tasks``); each request's thief duration is ``get_task_duration +
    get_comm_cost(ts, thief)`` from the problem arrays; the victim duration is the device's
    ``st_cost`` (the same two terms). Messages go per victim in request order (one
    ``BatchedSend.send(*msgs)``). Returns the ``("request", log)`` entries."""
    st_task = np.asarray(out["st_task"], np.int64)
    if not len(st_task):
        return []
    # the bulk allocations (in-flight records, messages, log entries) would trigger the cyclic
    # collector again and again over the scheduler's whole heap; none of them forms a cycle
    was = gc.isenabled()
    gc.disable()
    try:
        return _apply_requests(plugin, out, p, rows, wss, start, st_task)
    finally:
        if was:
            gc.enable()


def _apply_requests(plugin, out, p, rows, wss, start, st_task) -> list:
    s = plugin.scheduler
    K = len(st_task)
    slots = np.asarray(rows)[st_task]
    tss = _gather(plugin.rows.task, slots.tolist())
    vi, ti = np.asarray(out["st_victim"], np.int64), np.asarray(out["st_thief"], np.int64)
    lv = np.asarray(out["st_level"], np.int64)
    cost = np.asarray(out["st_cost"], np.float64)
    thief_dur = np.asarray(p["duration"], np.float64)[st_task] + thief_comm_bytes(p, st_task, ti) / s.bandwidth
    c0 = plugin._request_counter
    plugin._request_counter = c0 + K
    sids = [f"steal-{c}" for c in range(c0, c0 + K)]
    A = [ws.address for ws in wss]
    per_victim = [None] * len(wss)
    ks_pop, bins, slot_pop = plugin.key_stealable.pop, plugin.stealable, plugin.rows.slot.pop
    inflight = plugin.in_flight
    log = []
    log_append = log.append
    # one pass over the requests, each TaskState touched once: its bin (remove_key_from_stealable
    # :230-239), its row slot, the steal-request message (:306-308), the in-flight record
    # (:309-320, _add_to_in_flight :192) and the log entry (:468-478)
    for ts, sid, w, t_, l_, c, vd, td, ov, ot in zip(tss, sids, vi.tolist(), ti.tolist(), lv.tolist(), cost.tolist(),
                                                     cost.tolist(), thief_dur.tolist(),
                                                     np.asarray(out["st_occ_victim"]).tolist(),
                                                     np.asarray(out["st_occ_thief"]).tolist()):
        r = ks_pop(ts, None)
        if r is not None:
            bins[r[0]][r[1]].discard(ts)
        slot_pop(ts, None)
        key = ts.key
        m = per_victim[w]
        if m is None:
            m = per_victim[w] = []
        m.append({"op": "steal-request", "key": key, "stimulus_id": sid})
        v, t = wss[w], wss[t_]
        inflight[ts] = {"victim": v, "thief": t, "victim_duration": vd, "thief_duration": td, "stimulus_id": sid}
        log_append((start, l_, key, c, A[w], ov, A[t_], ot))
    plugin.rows.remove_many((), slots)  # the slots themselves (their TaskStates left above)
    comms = getattr(s, "stream_comms", {})
    for w, msgs in enumerate(per_victim):
        if msgs:
            comms[A[w]].send(*msgs)
    plugin._in_flight_event.clear()
    iocc, itsk = out["inflight_occ"], out["inflight_tasks"]
    io, it = plugin.in_flight_occupancy, plugin.in_flight_tasks
    for i in np.unique(np.concatenate([vi, ti])).tolist():
        io[wss[i]] = float(iocc[i])
        it[wss[i]] = int(itsk[i])
    # metrics (:479-480): counts per level, and the costs summed per level in request order
    # (np.cumsum adds sequentially, as the reference's += does)
    mc, mt = plugin.metrics["request_count_total"], plugin.metrics["request_cost_total"]
    for l_ in np.unique(lv).tolist():
        sel = cost[lv == l_]
        mc[l_] += int(len(sel))
        mt[l_] = float(np.cumsum(np.concatenate([[mt[l_]], sel]))[-1])
    return log

def _gather(seq, idx):
    """[seq[i] for i in idx] in one C call (operator.itemgetter); a tuple."""
    if not idx:
        return ()
    if len(idx) == 1:
        return (seq[idx[0]],)
    return operator.itemgetter(*idx)(seq)

def balance_plan(plugin, engine):
    """GPUWorkStealing.balance()'s decisions from the plugin's state, before any of them is
    applied: (device outputs, each output row's StealRows slot, workers in device order), or
    None for balance()'s early exits (stealing.py:409-411). ``plugin``: the plugin (or a
    stand-in with its attributes: scheduler, rows, in_flight_occupancy / in_flight_tasks)."""
    s = plugin.scheduler
    if not s.idle or len(s.idle) == len(s.workers):
        return None
    p, rows, wss = plugin.rows.problem(plugin)
    out = engine.steal_balance(p)
    plugin._last_problem = p  # apply_requests reads its dependency rows (thief durations)
    return out, rows, wss


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


def _restriction_rows(p, s, at, T, widx) -> None:
    """valid_workers (scheduler.py:3043-3107) of the restricted tasks, read at balance time.
    ``at``: (problem position, TaskState) of the tasks that may be restricted."""
    flags = np.zeros(T, np.uint8)
    vrows = {}
    for i, ts in at:
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

    def __init__(self, scheduler, *, device: int = 0, engine_factory=None, validate: bool = False,
                 bulk: bool = True):
        self.device = device
        self.engine_factory = engine_factory
        self.validate = validate
        self.bulk = bulk  # requests applied in bulk (apply_requests); False: move_task_request each
        self.engine = None
        self.gpu_stats = Counter()
        self.rows = StealRows()  # before the reference __init__: its hooks may fill the bins
        super().__init__(scheduler)
        self._wrap_replicas()

    def _wrap_replicas(self):
        """who_has of the dependencies in the rows follows SchedulerState.add_replica /
        remove_replica / remove_all_replicas (scheduler.py:3148-3171; every replica change
        goes through them), so balance() reads no TaskState."""
        s = self.scheduler
        add, rem, clr = (getattr(s, n, None) for n in ("add_replica", "remove_replica", "remove_all_replicas"))
        if add is None or rem is None or clr is None or getattr(s, "_gpu_steal_replicas", None) is self:
            return

        def add_replica(ts, ws):
            r = add(ts, ws)
            self.rows.replica(ts, ws.address, +1)
            return r

        def remove_replica(ts, ws):
            r = rem(ts, ws)
            self.rows.replica(ts, ws.address, -1)
            return r

        def remove_all_replicas(ts):
            r = clr(ts)
            self.rows.replicas_cleared(ts)
            return r

        s.add_replica, s.remove_replica, s.remove_all_replicas = add_replica, remove_replica, remove_all_replicas
        s._gpu_steal_replicas = self

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

    def _rows_current(self):
        """The rows, rebuilt from the bins if anything changed the bins outside the hooks."""
        if len(self.rows) != len(self.key_stealable):
            self.gpu_stats["rows_rebuilt"] += 1
            self.rows.clear()
            for ts, (worker, level) in self.key_stealable.items():
                self.rows.put(ts, worker, level)
        return self.rows

    def problem(self):
        """The dgp_steal_balance inputs of the current state: (problem, row slots, workers)."""
        return self._rows_current().problem(self)

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
        self._rows_current()
        plan = balance_plan(self, self._engine())  # the early exits of balance() (:409-411) inside
        if plan is None:
            return
        out, rows, wss = plan
        if self.bulk and self._comms_open(out, wss):
            log = apply_requests(self, out, self._last_problem, rows, wss, start)
        else:
            log = self._apply_one_by_one(out, rows, wss, start)
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

    def _comms_open(self, out, wss) -> bool:
        """Every victim's stream is open: a closed one makes move_task_request skip that
        request's in-flight record (:322-324), which only the per-request path restates."""
        comms = getattr(self.scheduler, "stream_comms", {})
        for i in np.unique(np.asarray(out["st_victim"])).tolist():
            c = comms.get(wss[i].address)
            comm = getattr(c, "comm", None)
            if c is None or (comm is not None and comm.closed()):
                return False
        return True

    def _apply_one_by_one(self, out, rows, wss, start) -> list:
        """The requests through the reference's own ``move_task_request``, one at a time."""
        task = self.rows.task
        slots = rows[out["st_task"]].tolist()
        log = []
        for k, sl in enumerate(slots):
            ts = task[sl]
            victim, thief = wss[int(out["st_victim"][k])], wss[int(out["st_thief"][k])]
            level = int(out["st_level"][k])
            cost = float(out["st_cost"][k])
            self.move_task_request(ts, victim, thief)  # :466
            log.append((start, level, ts.key, cost, victim.address, float(out["st_occ_victim"][k]), thief.address,
                        float(out["st_occ_thief"][k])))
            self.metrics["request_count_total"][level] += 1  # :479-480
            self.metrics["request_cost_total"][level] += cost
        return log

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
