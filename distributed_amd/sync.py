"""The scheduler's placement state as the engine's resync rows (``dgp_sync_*``,
``include/dgplace.h``).

After a stimulus the engine does not model (a worker removed, a rescheduled task, a client
releasing keys, ...) the extension lets the scheduler decide that one stimulus itself and
then hands the engine the state the scheduler ended in, read from the reference's own
objects (``distributed/scheduler.py``): ``TaskState`` (:1173-1540: state, waiting_on,
waiters, processing_on, nbytes, who_has, who_wants), ``WorkerState`` (:406-845: status,
processing, long_running, task_prefix_count, _network_occ, nbytes, needs_what),
``SchedulerState`` (idle, saturated, n_tasks, _network_occ_global,
_task_prefix_count_global, queued, bandwidth, total_nthreads), ``TaskPrefix``
(duration_average, max_exec_time :923-1031) and ``TaskGroup`` (states, last_worker,
last_worker_tasks_left :1033-1170).

Pure Python over duck-typed scheduler objects (no dask import): the extension calls it on
the live scheduler, ``tests/golden/gen_service.py`` on the reference replay state.
"""
from __future__ import annotations

import numpy as np

STATE_CODES = {"released": 0, "waiting": 1, "processing": 2, "queued": 3, "no-worker": 4, "memory": 5, "erred": 6,
               "forgotten": 7}
PD = 8  # task_prefix_count entries per worker the engine carries (dgp_stream.h PD)


def task_rows(s, keys, task_index, worker_index) -> dict:
    """Rows of ``dgp_sync_tasks`` for ``keys`` (tasks of the engine's graph)."""
    n = len(keys)
    out = dict(task=np.zeros(n, np.int32), state=np.zeros(n, np.uint8), remaining=np.zeros(n, np.int32),
               waiters=np.zeros(n, np.int32), processing_on=np.full(n, -1, np.int32),
               nbytes=np.full(n, -1, np.int64), long_running=np.zeros(n, np.uint8), wanted=np.zeros(n, np.uint8),
               holder_ptr=np.zeros(n + 1, np.int64))
    holders = []
    for i, key in enumerate(keys):
        out["task"][i] = task_index[key]
        ts = s.tasks.get(key)
        if ts is None:  # forgotten: gone from SchedulerState.tasks and from its dependencies' dependents
            out["state"][i] = STATE_CODES["forgotten"]
            out["holder_ptr"][i + 1] = len(holders)
            continue
        out["state"][i] = STATE_CODES[ts.state]
        out["remaining"][i] = len(ts.waiting_on or ()) if ts.state == "waiting" else 0
        out["waiters"][i] = len(ts.waiters or ())
        ws = ts.processing_on
        if ts.state == "processing" and ws is not None:
            out["processing_on"][i] = worker_index[ws.address]
            out["long_running"][i] = 1 if ts in ws.long_running else 0
        out["nbytes"][i] = ts.nbytes
        out["wanted"][i] = 1 if ts.who_wants else 0
        holders.extend(sorted(worker_index[h.address] for h in (ts.who_has or ())))
        out["holder_ptr"][i + 1] = len(holders)
    out["holder_idx"] = np.array(holders, np.int32)
    return out


def worker_rows(s, workers, prefix_index, task_index) -> dict:
    """Rows of ``dgp_sync_workers``: ``workers`` lists the engine's worker addresses by index
    (a removed worker keeps its index and reads status 2)."""
    W = len(workers)
    out = dict(status=np.zeros(W, np.int8), nproc=np.zeros(W, np.int32), n_long_running=np.zeros(W, np.int32),
               plen=np.zeros(W, np.int32), prefix=np.zeros(W * PD, np.int32), count=np.zeros(W * PD, np.int32),
               netocc=np.zeros(W, np.int64), nbytes=np.zeros(W, np.int64), idle=np.zeros(W, np.uint8),
               saturated=np.zeros(W, np.uint8), needs_ptr=np.zeros(W + 1, np.int64))
    sat = {ws.address for ws in s.saturated}
    nt, nc = [], []
    for w, addr in enumerate(workers):
        ws = s.workers.get(addr)
        if ws is None:
            out["status"][w] = 2
            out["needs_ptr"][w + 1] = len(nt)
            continue
        out["status"][w] = 0 if ws in s.running else 1
        out["nproc"][w] = len(ws.processing)
        out["n_long_running"][w] = len(ws.long_running)
        items = list(ws.task_prefix_count.items())
        if len(items) > PD:
            raise NotImplementedError(f"{addr}: more than {PD} task prefixes processing")
        out["plen"][w] = len(items)
        for i, (name, cnt) in enumerate(items):
            out["prefix"][w * PD + i] = prefix_index[name]
            out["count"][w * PD + i] = cnt
        out["netocc"][w] = ws._network_occ
        out["nbytes"][w] = ws.nbytes
        out["idle"][w] = 1 if addr in s.idle else 0
        out["saturated"][w] = 1 if addr in sat else 0
        for ts, cnt in ws.needs_what.items():
            if ts.key not in task_index:
                raise NotImplementedError(f"{addr} needs {ts.key!r}, a task outside the engine's graph")
            nt.append(task_index[ts.key])
            nc.append(cnt)
        out["needs_ptr"][w + 1] = len(nt)
    out["needs_task"] = np.array(nt, np.int32)
    out["needs_count"] = np.array(nc, np.int32)
    return out


def global_rows(s, prefix_names, prefix_default, group_names, task_index, worker_index) -> dict:
    """``dgp_sync_globals``: the scheduler-wide quantities, in the engine's prefix / group
    table orders (``prefix_default``: a prefix the scheduler no longer knows keeps it)."""
    pidx = {nm: i for i, nm in enumerate(prefix_names)}
    gp = list(s._task_prefix_count_global.items())
    dur, mx = [], []
    for nm, d0 in zip(prefix_names, prefix_default):
        tp = s.task_prefixes.get(nm)
        dur.append(float(tp.duration_average) if tp is not None else float(d0))
        mx.append(float(tp.max_exec_time) if tp is not None else -1.0)
    G = len(group_names)
    relw, left, lastw = np.zeros(G, np.int64), np.zeros(G, np.int64), np.full(G, -1, np.int32)
    for g, nm in enumerate(group_names):
        tg = s.task_groups.get(nm)
        if tg is None:
            continue
        relw[g] = tg.states["released"] + tg.states["waiting"]
        left[g] = tg.last_worker_tasks_left
        if tg.last_worker is not None:
            lastw[g] = worker_index.get(tg.last_worker.address, -1)
    return dict(n_tasks=int(s.n_tasks), network_occ_global=float(s._network_occ_global),
                g_prefix=np.array([pidx[nm] for nm, _ in gp], np.int32), g_count=np.array([c for _, c in gp], np.int64),
                queued=np.array([task_index[ts.key] for ts in s.queued.sorted()], np.int32),
                duration_average=np.array(dur, np.float64), max_exec_time=np.array(mx, np.float64),
                bandwidth=float(s.bandwidth), group_released_waiting=relw, group_left=left, group_last_worker=lastw)


def placement_record(s, ts, ws, route: int) -> tuple:
    """What ``dgp_sync_placements`` logs for a placement the scheduler made
    (``_add_to_processing`` :3199, before it mutates): worker_objective's comm bytes
    (:3136-3138) and start time (:3140-3141), ws.nbytes and the decide_worker route."""
    comm = sum(d.get_nbytes() for d in ts.dependencies if ws not in (d.who_has or ()))
    start = ws.occupancy / ws.nthreads + comm / s.bandwidth
    return comm, start, ws.nbytes, route
