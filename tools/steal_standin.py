"""A scheduler-free stand-in of a WorkStealing plugin's state (bench.py's C4 balance() leg).

``GPUWorkStealing.balance()`` (distributed_amd/stealing.py) reads the plugin's own state --
its stealable bins as ``StealRows`` (filled by the transition hooks, stealing.py:218-239),
the in-flight accounts -- and a few scheduler fields (workers, idle / saturated, totals,
bandwidth, get_task_duration / valid_workers). The GPU box has no ``distributed``, so the
bench builds these from a C4 problem (graphs.steal_problem) with plain objects carrying
exactly the attributes balance() reads, fills the rows through ``StealRows.put`` as the
hooks would, with the reference plugin's bins (``stealable`` / ``key_stealable``) and
in-flight fields, and times ``GPUWorkStealing.balance``'s product path on it:
``balance_plan`` (plugin state to the ordered request arrays) and ``apply_requests`` (the
requests applied in bulk: bins, messages, in-flight records and accounts, log, metrics).
Test / bench scaffolding (tools/, not the product package).
"""
from __future__ import annotations

import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.stealing import StealRows  # noqa: E402


class Obj:
    """An attribute bag hashed by identity, like TaskState / WorkerState / TaskPrefix."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class Comm:
    """BatchedSend's send(*msgs) (batched.py:150-159), buffering."""

    def __init__(self):
        self.buffer = []
        self.comm = None

    def send(self, *msgs):
        self.buffer.extend(msgs)


class Event:
    def clear(self):
        pass

    def set(self):
        pass


class Sched:
    """The SchedulerState fields balance() reads."""

    def __init__(self, workers, idle, saturated, total_occupancy, total_nthreads, bandwidth):
        self.workers = workers
        self.idle = idle
        self.saturated = saturated
        self.total_occupancy = total_occupancy
        self.total_nthreads = total_nthreads
        self.bandwidth = bandwidth
        self.unknown_durations = {}
        self.stream_comms = {a: Comm() for a in workers}

    def get_task_duration(self, ts):  # scheduler.py:3024-3041
        d = ts.prefix.duration_average
        if d >= 0:
            return d
        self.unknown_durations.setdefault(ts.prefix.name, set()).add(ts)
        return 0.5

    def valid_workers(self, ts):
        return {self.workers[a] for a in ts.worker_restrictions if a in self.workers}


def _data(nbytes, get_nbytes, who_has):
    return Obj(nbytes=int(nbytes), who_has=who_has, get_nbytes=lambda v=int(get_nbytes): v)


def plugin_from_problem(p: dict, levels) -> tuple:
    """(plugin stand-in, task index of each StealRows slot) for the C4 problem ``p`` whose
    tasks sit in the bins ``levels`` give (-1: not stealable, not put). Task t's priority is
    (0, 1, t): the problem's own walk order."""
    W, T = len(p["nthreads"]), len(p["victim"])
    addr = [f"tcp://w{i:05d}:1" for i in range(W)]
    workers = {a: Obj(address=a, nthreads=int(p["nthreads"][i]), occupancy=float(p["occ"][i]),
                      processing=range(int(p["nproc"][i])), nbytes=int(p["wnbytes"][i]))
               for i, a in enumerate(addr)}
    wl = list(workers.values())
    s = Sched(workers, {addr[i]: wl[i] for i in np.flatnonzero(p["idle"]).tolist()},
              {wl[i] for i in np.flatnonzero(p["sat"]).tolist()}, float(p["total_occ"]), int(p["total_nthreads"]),
              int(p["bandwidth"]))
    if "holder_ptr" in p:
        hp, hi = p["holder_ptr"], p["holder_idx"]
        holders = [hi[hp[d]:hp[d + 1]] for d in range(len(hp) - 1)]
    else:
        holders = [[h] if h >= 0 else [] for h in p["data_holder"].tolist()]
    data = [_data(nb, gnb, {wl[int(h)] for h in hs})
            for nb, gnb, hs in zip(p["data_nbytes"].tolist(), p["data_get_nbytes"].tolist(), holders)]
    prefixes = {d: Obj(name=f"p{j}", duration_average=float(d)) for j, d in enumerate(sorted(set(p["duration"].tolist())))}
    plugin = Obj(scheduler=s, rows=StealRows(), in_flight_occupancy=defaultdict(int), in_flight_tasks=defaultdict(int),
                 in_flight={}, _request_counter=0, _in_flight_event=Event(), key_stealable={},
                 stealable={a: [set() for _ in range(15)] for a in addr},
                 metrics={"request_count_total": defaultdict(int), "request_cost_total": defaultdict(float)})
    dp, di = p["dep_ptr"], p["dep_idx"]
    lv = np.asarray(levels)
    slot_task = []
    for t in range(T):
        if lv[t] < 0:
            continue
        ts = Obj(key=("t", t), priority=(0, 1, t), dependencies=[data[int(d)] for d in di[dp[t]:dp[t + 1]]],
                 prefix=prefixes[float(p["duration"][t])], worker_restrictions=None, host_restrictions=None,
                 resource_restrictions=None, loose_restrictions=False)
        a, level = addr[int(p["victim"][t])], int(lv[t])
        plugin.stealable[a][level].add(ts)  # put_key_in_stealable (stealing.py:220-228)
        plugin.key_stealable[ts] = (a, level)
        plugin.rows.put(ts, a, level)
        slot_task.append(t)
    return plugin, np.array(slot_task, np.int64)
