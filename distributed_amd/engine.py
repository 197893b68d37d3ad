"""Host wrapper of the HIP placement engine (``libdgplace.so``).

``PlacementEngine`` owns one device engine. It takes a graph dict
(``distributed_amd/graphs.py``) and the scheduler knobs of ``distributed.yaml``,
keeps the graph resident in HBM and replays the reference placement path on the GPU.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


DEFAULT_CONFIG = {  # distributed/distributed.yaml:13,16,24,28
    "bandwidth": 100_000_000,
    "default_data_size": 1024,
    "unknown_duration": 0.5,
    "saturation": 1.1,
}

# ids of dgp_kernel_times; id 2 is the persistent replay kernel (k_stream; k_replay when P > PD);
# 4..6 are WorkStealing (levels + bins, thief argmin, balance walk)
KERNEL_NAMES = ("frontier_release", "candidate_commbytes", "replay", "update_graph", "steal_levels",
                "steal_thief_argmin", "steal_balance", "unused")


def conflict_depth(g: dict, out: dict, first: int = 0) -> tuple[int, int]:
    """(depth, touches): the longest chain of ordered stimuli in a replay's placement log
    (``dgp_conflict_depth``), from stimulus ``first`` on; the critical path of the latency
    bound bench.py reports."""
    lib = _lib.load()
    dp = np.ascontiguousarray(g["dep_ptr"], np.int64)
    di = np.ascontiguousarray(g["dep_idx"], np.int32)
    wa = np.ascontiguousarray(g["wanted"], np.uint8)
    pt = np.ascontiguousarray(out["pl_task"], np.int32)
    pw = np.ascontiguousarray(out["pl_worker"], np.int32)
    d, t = C.c_int64(0), C.c_int64(0)
    rc = lib.dgp_conflict_depth(int(g["n_tasks"]), _ptr(dp), _ptr(di), _ptr(wa), len(pt), _ptr(pt), _ptr(pw),
                                int(first), C.byref(d), C.byref(t))
    if rc != 0:
        raise _lib.DgpError(f"dgp_conflict_depth: status {rc}")
    return int(d.value), int(t.value)


class PlacementEngine:
    """One device engine bound to HIP device ``device``."""

    def __init__(self, device: int = 0, window: int | str = "auto"):
        """``window``: the stream kernel's in-flight stimulus window -- 32 (wait-in-place
        claims), 64 (no wait-in-place) or "auto": chosen per graph by ``auto_window`` at
        ``load`` and at each later graph (the unpacks' completions after a wide
        frontier are window-bound; the C2 chain needs wait-in-place). Both builds are in the
        one library (``dgp_set_window``) and make identical placements."""
        if window not in (*_lib.WINDOWS, "auto"):
            raise ValueError(f"window must be 32, 64 or 'auto', not {window!r}")
        self.window = window
        self.lib = _lib.load()
        self.device = int(device)
        h = self.lib.dgp_create(int(device))
        if not h:
            raise _lib.DgpError(f"dgp_create({device}) failed: no HIP device visible (no CPU fallback)")
        self.h = h
        if window != "auto":
            self.set_window(window)
        self.n_tasks = 0
        self.n_workers = 0
        self._keep = []
        self._posted_n = 0
        # per-call buffers of the extension's service path (tasks_finished_post / _wait, answer)
        self._one = None
        self._st = np.zeros(64, np.int8)
        self._st_ptr = _ptr(self._st)
        self._newp, self._nd, self._nh = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        self._newp_ref, self._nd_ref, self._nh_ref = C.byref(self._newp), C.byref(self._nd), C.byref(self._nh)
        self._ans = None

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.dgp_last_error(self.h)
            raise _lib.DgpError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.dgp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------------- set-up
    def set_config(self, config: dict | None = None):
        cfg = dict(DEFAULT_CONFIG, **(config or {}))
        sat = cfg["saturation"]
        sat = math.inf if sat == "inf" else float(sat)
        self._check(self.lib.dgp_set_config(self.h, int(cfg["bandwidth"]), int(cfg["default_data_size"]),
                                            float(cfg["unknown_duration"]), sat), "dgp_set_config")
        self.config = cfg

    def set_workers(self, nthreads):
        nt = np.ascontiguousarray(nthreads, dtype=np.int32)
        self._check(self.lib.dgp_set_workers(self.h, len(nt), _ptr(nt)), "dgp_set_workers")
        self.n_workers = len(nt)

    def set_graph(self, g: dict, results: bool = True):
        arrs = {
            "dep_ptr": np.ascontiguousarray(g["dep_ptr"], np.int64),
            "dep_idx": np.ascontiguousarray(g["dep_idx"], np.int32),
            "prio": np.ascontiguousarray(g["prio"], np.int64),
            "prefix_id": np.ascontiguousarray(g["prefix_id"], np.int32),
            "prefix_default_dur": np.ascontiguousarray(g["prefix_default_dur"], np.float64),
            "group_id": np.ascontiguousarray(g["group_id"], np.int32),
            "wanted": np.ascontiguousarray(g["wanted"], np.uint8),
            "rootish_override": np.ascontiguousarray(g["rootish_override"], np.int8),
        }
        n = len(arrs["prio"])
        self._check(self.lib.dgp_set_graph(
            self.h, n, _ptr(arrs["dep_ptr"]), _ptr(arrs["dep_idx"]), _ptr(arrs["prio"]), _ptr(arrs["prefix_id"]),
            len(arrs["prefix_default_dur"]), _ptr(arrs["prefix_default_dur"]), _ptr(arrs["group_id"]),
            len(g["group_prefix"]), _ptr(arrs["wanted"]), _ptr(arrs["rootish_override"])), "dgp_set_graph")
        self.n_tasks = n
        if g.get("restr_flags") is not None:  # worker restrictions, resolved (graphs.restrict)
            r = [np.ascontiguousarray(g["restr_ptr"], np.int64), np.ascontiguousarray(g["restr_idx"], np.int32),
                 np.ascontiguousarray(g["restr_flags"], np.uint8)]
            self._check(self.lib.dgp_set_restrictions(self.h, *[_ptr(a) for a in r]), "dgp_set_restrictions")
        if not results:  # service mode: the task-finished messages carry nbytes / startstops
            return
        res = [np.ascontiguousarray(g["nbytes"], np.int64), np.ascontiguousarray(g["start"], np.float64),
               np.ascontiguousarray(g["stop"], np.float64)]
        self._check(self.lib.dgp_set_task_results(self.h, *[_ptr(a) for a in res]), "dgp_set_task_results")

    def load(self, g: dict, config: dict | None = None, *, snapshots: int = 0, results: bool = True):
        """Configure workers + config + graph in one go (the usual set-up). ``results``:
        upload the synthetic executor's completion reports (replay mode)."""
        if self.window == "auto":
            self.set_window(self.auto_window(g))
        self.set_workers(g["nthreads"])
        self.set_config(config)
        if snapshots:
            self._check(self.lib.dgp_enable_snapshots(self.h, int(snapshots)), "dgp_enable_snapshots")
        self.set_graph(g, results=results)
        return self

    WIDE_FRONTIER = 4096  # dependents of one task from which the 64-slot build is chosen

    @classmethod
    def auto_window(cls, g: dict) -> int:
        """64 for a graph with restrictions or a wide frontier (a task with at least
        WIDE_FRONTIER dependents: the P2P barrier, whose completion readies every unpack at
        once), else 32."""
        rf = g.get("restr_flags")
        if rf is not None and np.asarray(rf).any():
            return 64
        di = np.asarray(g["dep_idx"])
        if len(di) and int(np.bincount(di[di >= 0]).max()) >= cls.WIDE_FRONTIER:
            return 64
        return 32

    def set_window(self, window: int):
        """The stream kernel build the next launches run (32 or 64 slots, ABI 19)."""
        self._check(self.lib.dgp_set_window(self.h, int(window)), "dgp_set_window")

    def get_window(self) -> int:
        return int(self.lib.dgp_get_window(self.h))

    def later_graph_window(self, g: dict):
        """A later graph on an "auto" engine: the 64-slot build from the first graph that
        wants it (restrictions or a wide frontier) on; a 32-slot engine stays unless so."""
        if self.window == "auto" and self.get_window() != 64 and self.auto_window(g) == 64:
            self.set_window(64)

    # ------------------------------------------------------------------- replay
    def reset(self):
        self._check(self.lib.dgp_reset(self.h), "dgp_reset")

    def update_graph(self):
        self._check(self.lib.dgp_update_graph(self.h), "dgp_update_graph")

    def run_rounds(self, max_rounds: int = -1) -> int:
        n = C.c_int64(0)
        self._check(self.lib.dgp_run_rounds(self.h, int(max_rounds), C.byref(n)), "dgp_run_rounds")
        return int(n.value)

    def replay(self) -> int:
        """update_graph + every round; returns the number of placements."""
        self.update_graph()
        self.run_rounds(-1)
        return self.num_placements()

    # ------------------------------------------------------------- service mode
    # answers of dgp_tasks_finished (include/dgplace.h DGP_TF_*)
    TF_ACCEPTED, TF_FREE_KEYS, TF_ADD_KEYS, TF_RELEASE, TF_UNKNOWN_WORKER, TF_IMPOSSIBLE, TF_UNSUPPORTED = range(7)

    @staticmethod
    def _tf_batch(task, worker, run_id, nbytes, start, stop):
        t = np.ascontiguousarray(task, np.int32).reshape(-1)
        n = len(t)
        w = np.ascontiguousarray(worker, np.int32).reshape(-1)
        r = np.ascontiguousarray(run_id, np.int64).reshape(-1)
        nb = np.ascontiguousarray(np.full(n, -1) if nbytes is None else nbytes, np.int64).reshape(-1)
        a = np.ascontiguousarray(np.full(n, np.nan) if start is None else start, np.float64).reshape(-1)
        b = np.ascontiguousarray(np.full(n, np.nan) if stop is None else stop, np.float64).reshape(-1)
        if not (len(w) == len(r) == len(nb) == len(a) == len(b) == n):
            raise ValueError("tasks_finished: all message fields need the same length")
        return n, (t, w, r, nb, a, b)

    def tasks_finished(self, task, worker, run_id, nbytes=None, start=None, stop=None):
        """A batch of task-finished messages (Scheduler.handle_task_finished,
        distributed/scheduler.py:5783-5797), in arrival order. ``nbytes`` < 0 means None;
        ``start``/``stop`` is the "compute" startstop (NaN: none). Returns (status per
        message, number of placements the batch made)."""
        n, cols = self._tf_batch(task, worker, run_id, nbytes, start, stop)
        st = np.zeros(n, np.int8)
        newp = C.c_int64(0)
        self._check(self.lib.dgp_tasks_finished(self.h, n, *map(_ptr, cols), _ptr(st), C.byref(newp)),
                    "dgp_tasks_finished")
        return st, int(newp.value)

    def tasks_finished_post(self, task, worker, run_id, nbytes=None, start=None, stop=None):
        """The first half of ``tasks_finished`` (dgp_tasks_finished_post): the batch goes to
        the device and the call returns; ``tasks_finished_wait`` takes the answer. In
        between, the caller's own work runs while the device decides. A one-message batch
        goes through preallocated buffers (the extension's per-message case)."""
        if len(task) == 1 and nbytes is not None and start is not None and stop is not None:
            one = self._one
            if one is None:
                one = self._one = tuple(np.zeros(1, dt) for dt in (np.int32, np.int32, np.int64, np.int64,
                                                                    np.float64, np.float64))
                self._one_ptrs = tuple(_ptr(x) for x in one)
            one[0][0], one[1][0], one[2][0], one[3][0], one[4][0], one[5][0] = (
                task[0], worker[0], run_id[0], nbytes[0], start[0], stop[0])
            rc = self.lib.dgp_tasks_finished_post(self.h, 1, *self._one_ptrs)
            n = 1
        else:
            n, cols = self._tf_batch(task, worker, run_id, nbytes, start, stop)
            rc = self.lib.dgp_tasks_finished_post(self.h, n, *map(_ptr, cols))
        self._check(rc, "dgp_tasks_finished_post")
        self._posted_n = n

    def tasks_finished_wait(self):
        """(status per message, number of new placements) of the posted batch."""
        n = self._posted_n
        if n > len(self._st):
            self._st = np.zeros(max(n, 2 * len(self._st)), np.int8)
            self._st_ptr = _ptr(self._st)
        self._check(self.lib.dgp_tasks_finished_wait(self.h, self._st_ptr, self._newp_ref), "dgp_tasks_finished_wait")
        return self._st[:n].copy(), int(self._newp.value)

    @staticmethod
    def _ans_grow(b, d, h):
        if d > b["dcap"]:
            b["dcap"] = max(d, 2 * b["dcap"])
            b.update(dt=np.zeros(b["dcap"], np.int32), dn=np.zeros(b["dcap"], np.int64),
                     hp=np.zeros(b["dcap"] + 1, np.int64))
            b.update(pdt=_ptr(b["dt"]), pdn=_ptr(b["dn"]), php=_ptr(b["hp"]))
        if h > b["hcap"]:
            b["hcap"] = max(h, 2 * b["hcap"])
            b["hi"] = np.zeros(b["hcap"], np.int32)
            b["phi"] = _ptr(b["hi"])

    def answer(self, offset: int, count: int, messages: bool = True):
        """What the extension takes after an answer, in one go and as Python lists: the task
        and worker of placements [offset, offset + count) (dgp_get_placements) and, with
        ``messages``, their compute-task fields (dgp_task_messages: dep_ptr, dep_task,
        dep_nbytes, holder_ptr, holder_idx) -- or None. Preallocated buffers, no numpy
        allocation per call."""
        b = self._ans
        if b is None or b["cap"] < count:
            cap = max(count, 64, 2 * (b["cap"] if b else 0))
            b = self._ans = dict(cap=cap, pt=np.zeros(cap, np.int32), pw=np.zeros(cap, np.int32),
                                 dp=np.zeros(cap + 1, np.int64), dcap=0, hcap=0)
            b.update(ppt=_ptr(b["pt"]), ppw=_ptr(b["pw"]), pdp=_ptr(b["dp"]))
            self._ans_grow(b, 256, 256)
        self._check(self.lib.dgp_get_placements(self.h, offset, count, b["ppt"], b["ppw"], None, None, None, None),
                    "dgp_get_placements")
        tasks, workers = b["pt"][:count].tolist(), b["pw"][:count].tolist()
        if not messages:
            return tasks, workers, None
        nd, nh = self._nd, self._nh
        self._check(self.lib.dgp_task_messages(self.h, offset, count, self._nd_ref, self._nh_ref, None, None, None,
                                               None, None), "dgp_task_messages")
        d, h = nd.value, nh.value
        if d > b["dcap"] or h > b["hcap"]:
            self._ans_grow(b, d, h)
        self._check(self.lib.dgp_task_messages(self.h, offset, count, self._nd_ref, self._nh_ref, b["pdp"], b["pdt"],
                                               b["pdn"], b["php"], b["phi"]), "dgp_task_messages")
        return tasks, workers, (b["dp"][:count + 1].tolist(), b["dt"][:d].tolist(), b["dn"][:d].tolist(),
                                b["hp"][:d + 1].tolist(), b["hi"][:h].tolist())

    def set_resident(self, on: bool = True):
        """Resident service mode (dgp_set_resident): the stream kernel stays launched between
        tasks_finished calls and takes each batch from a pinned mailbox."""
        self._check(self.lib.dgp_set_resident(self.h, 1 if on else 0), "dgp_set_resident")

    def set_task_messages(self, on: bool = True):
        """Resident answers carry their placements' compute-task message fields
        (dgp_set_task_messages): task_messages of the last answer reads the mailbox."""
        self._check(self.lib.dgp_set_task_messages(self.h, 1 if on else 0), "dgp_set_task_messages")

    def move_task(self, task: int, thief: int):
        """Steal confirmation (WorkStealing.move_task_confirm, distributed/stealing.py
        :376-384): processing ``task`` moves from its worker to ``thief`` on the device."""
        self._check(self.lib.dgp_move_task(self.h, int(task), int(thief)), "dgp_move_task")

    def add_worker(self, nthreads: int, *, running: bool = True, position: int | None = None) -> int:
        """A worker joins (Scheduler.add_worker, distributed/scheduler.py:4308-4441):
        check_idle_saturated and the queue refill on the device. ``position``: its index in
        the address order of the engine's workers (default: after all of them); every later
        worker's index moves up by one (dgp_add_worker_at). ``running`` False: it joins
        paused (no refill). Returns the number of placements the refill made."""
        newp = C.c_int64(0)
        pos = self.n_workers if position is None else int(position)
        self._check(self.lib.dgp_add_worker_at(self.h, int(nthreads), 1 if running else 0, pos, C.byref(newp)),
                    "dgp_add_worker_at")
        self.n_workers += 1
        return int(newp.value)

    def add_graph(self, g: dict, defer: bool = False) -> int:
        """A later graph submission (Scheduler.update_graph, distributed/scheduler.py
        :4662-4751) on a running engine: ``g`` holds the new tasks only (dependencies
        relative to it, ``-1 - t`` for an earlier task t; priorities after every earlier
        task's, prefix / group ids and ``prefix_default_dur`` / ``group_prefix`` over the
        engine-wide tables). Runs their update_graph stimulus; returns the number of
        placements it made. With dependencies on earlier tasks the stimulus is the
        scheduler's: nothing is placed and ``sync()`` must follow (include/dgplace.h); so
        too with ``defer`` (dgp_add_graph_deferred: a graph with restrictions)."""
        self.later_graph_window(g)
        arrs = {
            "dep_ptr": np.ascontiguousarray(g["dep_ptr"], np.int64),
            "dep_idx": np.ascontiguousarray(g["dep_idx"], np.int32),
            "prio": np.ascontiguousarray(g["prio"], np.int64),
            "prefix_id": np.ascontiguousarray(g["prefix_id"], np.int32),
            "prefix_default_dur": np.ascontiguousarray(g["prefix_default_dur"], np.float64),
            "group_id": np.ascontiguousarray(g["group_id"], np.int32),
            "wanted": np.ascontiguousarray(g["wanted"], np.uint8),
            "rootish_override": np.ascontiguousarray(g["rootish_override"], np.int8),
        }
        n = len(arrs["prio"])
        newp = C.c_int64(0)
        if defer:
            self._check(self.lib.dgp_add_graph_deferred(
                self.h, n, _ptr(arrs["dep_ptr"]), _ptr(arrs["dep_idx"]), _ptr(arrs["prio"]), _ptr(arrs["prefix_id"]),
                len(arrs["prefix_default_dur"]), _ptr(arrs["prefix_default_dur"]), _ptr(arrs["group_id"]),
                len(g["group_prefix"]), _ptr(arrs["wanted"]), _ptr(arrs["rootish_override"])), "dgp_add_graph_deferred")
            self.n_tasks += n
            return 0
        self._check(self.lib.dgp_add_graph(
            self.h, n, _ptr(arrs["dep_ptr"]), _ptr(arrs["dep_idx"]), _ptr(arrs["prio"]), _ptr(arrs["prefix_id"]),
            len(arrs["prefix_default_dur"]), _ptr(arrs["prefix_default_dur"]), _ptr(arrs["group_id"]),
            len(g["group_prefix"]), _ptr(arrs["wanted"]), _ptr(arrs["rootish_override"]), C.byref(newp)),
            "dgp_add_graph")
        self.n_tasks += n
        return int(newp.value)

    UNSUPPORTED = -5  # DGP_E_UNSUPPORTED: a case the engine leaves to the caller, nothing changed

    def graph_stimulus(self, order=None) -> int | None:
        """The update_graph stimulus of the graph ``add_graph(defer=True)`` appended, on the
        device (dgp_graph_stimulus): dependent, restricted (rows first, update_restrictions)
        or outranking (ranks first, set_priorities) later graphs. ``order``: (task, kind,
        tasks) rows of the set orders a recompute of released earlier dependencies follows
        (``distributed_amd.loss.graph_orders``; given, even empty, the engine recomputes
        them: dgp_graph_stimulus_ordered). Returns its placements, or None when the engine
        leaves it to the scheduler (an earlier dependency released without ``order``, erred
        or forgotten): then the scheduler's stimulus and ``sync()`` follow as before."""
        newp = C.c_int64(0)
        if order is not None:
            ot, ok, op, oi = self._order_rows(order)
            rc = self.lib.dgp_graph_stimulus_ordered(self.h, len(ot), _ptr(ot), _ptr(ok), _ptr(op), _ptr(oi),
                                                     C.byref(newp))
        else:
            rc = self.lib.dgp_graph_stimulus(self.h, C.byref(newp))
        if rc == self.UNSUPPORTED:
            self.refusal = (self.lib.dgp_last_error(self.h) or b"").decode()
            return None
        self._check(rc, "dgp_graph_stimulus")
        return int(newp.value)

    def set_priorities(self, prio):
        """Every task's priority anew (dgp_set_priorities): the merged ranks after a later
        graph whose user priority outranks earlier tasks (appended with ``defer``)."""
        p = np.ascontiguousarray(prio, np.int64).reshape(-1)
        if len(p) != self.n_tasks:
            raise ValueError(f"set_priorities: {len(p)} priorities for {self.n_tasks} tasks")
        self._check(self.lib.dgp_set_priorities(self.h, _ptr(p)), "dgp_set_priorities")

    def remap_prefixes(self, task_prefix, prefix_default_duration):
        """The task prefix table anew (dgp_remap_prefixes): every task's slot in a table of
        at most 32 live prefixes and each slot's default duration; ``sync(workers=...,
        globals_=...)`` in the new numbering must follow before any other stimulus."""
        t = np.ascontiguousarray(task_prefix, np.int32).reshape(-1)
        d = np.ascontiguousarray(prefix_default_duration, np.float64).reshape(-1)
        if len(t) != self.n_tasks:
            raise ValueError(f"remap_prefixes: {len(t)} slots for {self.n_tasks} tasks")
        self._check(self.lib.dgp_remap_prefixes(self.h, len(d), _ptr(t), _ptr(d)), "dgp_remap_prefixes")

    # --------------------------------------------------------- service events
    @staticmethod
    def _arr(x, dt):
        return np.ascontiguousarray(np.asarray(x, dtype=dt).reshape(-1))

    def add_replicas(self, task, worker):
        """SchedulerState.add_replica for each (task, worker) pair (distributed/scheduler.py
        :3148-3153), e.g. from the add-keys stream handler (:7359-7391)."""
        t, w = self._arr(task, np.int32), self._arr(worker, np.int32)
        self._check(self.lib.dgp_add_replicas(self.h, len(t), _ptr(t), _ptr(w)), "dgp_add_replicas")

    def remove_replicas(self, task, worker):
        """SchedulerState.remove_replica for each pair (:3155-3159), release-worker-data."""
        t, w = self._arr(task, np.int32), self._arr(worker, np.int32)
        self._check(self.lib.dgp_remove_replicas(self.h, len(t), _ptr(t), _ptr(w)), "dgp_remove_replicas")

    def set_worker_status(self, worker: int, running: int) -> int:
        """handle_worker_status_change (:5850-5883); returns the placements of the refill."""
        n = C.c_int64(0)
        self._check(self.lib.dgp_set_worker_status(self.h, int(worker), int(running), C.byref(n)),
                    "dgp_set_worker_status")
        return int(n.value)

    def long_running(self, task: int, compute_duration: float = math.nan) -> int:
        """handle_long_running (:5817-5848); NaN = compute_duration None."""
        n = C.c_int64(0)
        self._check(self.lib.dgp_long_running(self.h, int(task), float(compute_duration), C.byref(n)),
                    "dgp_long_running")
        return int(n.value)

    def heartbeat(self, bandwidth: float, prefixes=(), durations=()):
        """heartbeat_worker's bandwidth EWMA result and add_exec_time per executing task's
        prefix (:4223-4226, :4247-4252)."""
        p, d = self._arr(prefixes, np.int32), self._arr(durations, np.float64)
        if len(p) != len(d):
            raise ValueError("heartbeat: one duration per prefix")
        self._check(self.lib.dgp_heartbeat(self.h, float(bandwidth), len(p), _ptr(p), _ptr(d)), "dgp_heartbeat")

    def set_worker_flags(self, workers, idle, saturated):
        """idle / saturated membership of ``workers`` as the scheduler holds it."""
        w, a, b = self._arr(workers, np.int32), self._arr(idle, np.uint8), self._arr(saturated, np.uint8)
        self._check(self.lib.dgp_set_worker_flags(self.h, len(w), _ptr(w), _ptr(a), _ptr(b)), "dgp_set_worker_flags")

    def update_restrictions(self, task, rows, flags):
        """Scheduler.set_restrictions of ``task`` while the graph runs (scheduler.py
        :7702-7707; the shuffle's restrict_task, shuffle/_scheduler_plugin.py:101-115): each
        task's valid workers (ascending engine indices) and flags (1 restricted, 2 loose)."""
        t, f = self._arr(task, np.int32), self._arr(flags, np.uint8)
        rows = [sorted(int(w) for w in r) for r in rows]
        if len(rows) != len(t) or len(f) != len(t):
            raise ValueError("update_restrictions: one row and one flag per task")
        rp = np.zeros(len(t) + 1, np.int64)
        rp[1:] = np.cumsum([len(r) for r in rows])
        ri = self._arr([w for r in rows for w in r], np.int32)
        if len(ri) == 0:
            ri = np.zeros(1, np.int32)
        if self.window == "auto" and f.any() and self.get_window() != 64:
            self.set_window(64)  # restrictions from now on: the 64-slot build (auto_window)
        self._check(self.lib.dgp_update_restrictions(self.h, len(t), _ptr(t), _ptr(rp), _ptr(ri), _ptr(f)),
                    "dgp_update_restrictions")

    def set_rootish(self, task, value):
        """TaskState._rootish per task (-1 None, 0 False, 1 True), set while the graph runs
        (the shuffle's _ensure_output_tasks_are_non_rootish, shuffle/_scheduler_plugin.py
        :254-278)."""
        t, v = self._arr(task, np.int32), self._arr(value, np.int8)
        self._check(self.lib.dgp_set_rootish(self.h, len(t), _ptr(t), _ptr(v)), "dgp_set_rootish")

    def set_wanted(self, task, wanted):
        """who_wants non-empty (1) / empty (0) per task (client_desires_keys :5398-5415)."""
        t, f = self._arr(task, np.int32), self._arr(wanted, np.uint8)
        self._check(self.lib.dgp_set_wanted(self.h, len(t), _ptr(t), _ptr(f)), "dgp_set_wanted")

    def task_erred(self, task: int) -> int:
        """handle_task_erred (:5799-5805) of a current run with no retries left; returns the
        placements of the refill."""
        n = C.c_int64(0)
        self._check(self.lib.dgp_task_erred(self.h, int(task), C.byref(n)), "dgp_task_erred")
        return int(n.value)

    # ---------------------------------------------------------------- resync
    def remove_worker(self, worker: int):
        """Scheduler.remove_worker's worker table part (distributed/scheduler.py:5213-5231)."""
        self._check(self.lib.dgp_remove_worker(self.h, int(worker)), "dgp_remove_worker")

    def reschedule(self, task: int) -> int | None:
        """Scheduler._reschedule (distributed/scheduler.py:7900-7924) of a processing task on
        the device (dgp_reschedule): released from its worker, waiting again, placed again.
        Returns the placements it made (0 or 1), or None when the engine leaves it to the
        scheduler (a task nobody needs); then ``sync()`` follows as after remove_worker."""
        newp = C.c_int64(0)
        rc = self.lib.dgp_reschedule(self.h, int(task), C.byref(newp))
        if rc == self.UNSUPPORTED:
            self.refusal = (self.lib.dgp_last_error(self.h) or b"").decode()
            return None
        self._check(rc, "dgp_reschedule")
        return int(newp.value)

    def release_tasks(self, task, forget) -> int | None:
        """client-releases-keys (distributed/scheduler.py:5417-5430, dgp_release_tasks): the
        tasks its transitions reach in the scheduler's order (loss.release_plan), each released
        from its state -- a result with its replicas, cancelled work (processing, waiting,
        queued, no-worker) leaving its worker / the queue and its dependencies' waiters --
        forgotten where flagged, then the queue refill. Returns its placements, or None when the
        engine leaves it to the scheduler (an erred or forgotten task), with nothing changed."""
        t, f = self._arr(task, np.int32), self._arr(forget, np.uint8)
        if len(t) != len(f):
            raise ValueError("one forget flag per task")
        newp = C.c_int64(0)
        rc = self.lib.dgp_release_tasks(self.h, len(t), _ptr(t), _ptr(f), C.byref(newp))
        if rc == self.UNSUPPORTED:
            self.refusal = (self.lib.dgp_last_error(self.h) or b"").decode()
            return None
        self._check(rc, "dgp_release_tasks")
        return int(newp.value)

    @staticmethod
    def _order_rows(order):
        """(task, kind, tasks) rows as the C ABI's sorted CSR (one row per (task, kind): the first)."""
        rows, seen = [], set()
        for t, k, seq in order:
            if (int(t), int(k)) not in seen:
                seen.add((int(t), int(k)))
                rows.append((int(t), int(k), list(map(int, seq))))
        rows.sort()
        ot = np.array([r[0] for r in rows], np.int32)
        ok = np.array([r[1] for r in rows], np.int8)
        op = np.zeros(len(rows) + 1, np.int64)
        op[1:] = np.cumsum([len(r[2]) for r in rows]) if rows else []
        oi = np.array([x for r in rows for x in r[2]], np.int32)
        return ot, ok, op, oi

    def lose_worker(self, worker: int, processing, held, order=(), killed=None) -> int | None:
        """The whole Scheduler.remove_worker stimulus (distributed/scheduler.py:5180-5303) on
        the device (dgp_lose_worker_ordered): ``processing`` = the worker's processing tasks in
        the order the scheduler iterates them, ``held`` = its replicas in ws.has_what order,
        ``order`` = (task, kind, tasks) rows: the scheduler's iteration order of a task's
        dependencies (kind 0), waiters (kind 1) or dependents (kind 2) where the cascade
        follows a set (``distributed_amd.loss.loss_orders``), ``killed`` = a flag per
        processing task that ran out of retries (KilledWorker: erred at once). Returns the
        placements it made, or None when
        the engine leaves the stimulus to the scheduler (a cascade it does not restate);
        after a refusal from the device the scheduler's state follows by ``sync()`` as after
        remove_worker."""
        p, h = self._arr(processing, np.int32), self._arr(held, np.int32)
        ot, ok, op, oi = self._order_rows(order)
        kf = None if killed is None or not any(killed) else self._arr(killed, np.int8)
        if kf is not None and len(kf) != len(p):
            raise ValueError("killed: one flag per processing task")
        newp = C.c_int64(0)
        rc = self.lib.dgp_lose_worker_ordered(self.h, int(worker), len(p), _ptr(p), None if kf is None else _ptr(kf),
                                              len(h), _ptr(h), len(ot), _ptr(ot), _ptr(ok), _ptr(op), _ptr(oi),
                                              C.byref(newp))
        if rc == self.UNSUPPORTED:
            self.refusal = (self.lib.dgp_last_error(self.h) or b"").decode()
            return None
        self._check(rc, "dgp_lose_worker")
        return int(newp.value)

    def sync_placements(self, task, worker, comm, start, wsnbytes, route):
        """Append placements the scheduler made itself (their run identity: log position)."""
        a = [self._arr(task, np.int32), self._arr(worker, np.int32), self._arr(comm, np.int64),
             self._arr(start, np.float64), self._arr(wsnbytes, np.int64), self._arr(route, np.int8)]
        self._check(self.lib.dgp_sync_placements(self.h, len(a[0]), *[_ptr(x) for x in a]), "dgp_sync_placements")

    def sync_tasks(self, rows: dict):
        """``sync.task_rows`` -> dgp_sync_tasks."""
        k = ("task", "state", "remaining", "waiters", "processing_on", "nbytes", "long_running", "wanted",
             "holder_ptr", "holder_idx")
        dts = (np.int32, np.uint8, np.int32, np.int32, np.int32, np.int64, np.uint8, np.uint8, np.int64, np.int32)
        a = [self._arr(rows[n], d) for n, d in zip(k, dts)]
        self._check(self.lib.dgp_sync_tasks(self.h, len(a[0]), *[_ptr(x) for x in a]), "dgp_sync_tasks")

    def sync_workers(self, rows: dict):
        """``sync.worker_rows`` -> dgp_sync_workers."""
        k = ("status", "nproc", "n_long_running", "plen", "prefix", "count", "netocc", "nbytes", "idle", "saturated",
             "needs_ptr", "needs_task", "needs_count")
        dts = (np.int8, np.int32, np.int32, np.int32, np.int32, np.int32, np.int64, np.int64, np.uint8, np.uint8,
               np.int64, np.int32, np.int32)
        a = [self._arr(rows[n], d) for n, d in zip(k, dts)]
        self._check(self.lib.dgp_sync_workers(self.h, len(a[0]), *[_ptr(x) for x in a]), "dgp_sync_workers")

    def sync_globals(self, g: dict):
        """``sync.global_rows`` -> dgp_sync_globals."""
        gp, gc = self._arr(g["g_prefix"], np.int32), self._arr(g["g_count"], np.int64)
        q = self._arr(g["queued"], np.int32)
        da, mx = self._arr(g["duration_average"], np.float64), self._arr(g["max_exec_time"], np.float64)
        rw, lf = self._arr(g["group_released_waiting"], np.int64), self._arr(g["group_left"], np.int64)
        lw = self._arr(g["group_last_worker"], np.int32)
        self._check(self.lib.dgp_sync_globals(
            self.h, int(g["n_tasks"]), float(g["network_occ_global"]), len(gp), _ptr(gp), _ptr(gc), len(q), _ptr(q),
            _ptr(da), _ptr(mx), float(g["bandwidth"]), _ptr(rw), _ptr(lf), _ptr(lw)), "dgp_sync_globals")

    def sync(self, placements=None, tasks=None, workers=None, globals_=None):
        """The whole resync, in the order include/dgplace.h prescribes."""
        if placements is not None and len(placements["task"]):
            self.sync_placements(*(placements[k] for k in ("task", "worker", "comm", "start", "wsnbytes", "route")))
        if tasks is not None:
            self.sync_tasks(tasks)
        if workers is not None:
            self.sync_workers(workers)
        if globals_ is not None:
            self.sync_globals(globals_)

    def snapshot(self):
        """Append one per-worker snapshot (service mode round boundary)."""
        self._check(self.lib.dgp_snapshot(self.h), "dgp_snapshot")

    # ------------------------------------------------------------------ results
    def num_placements(self) -> int:
        n = self.lib.dgp_num_placements(self.h)
        if n < 0:
            self._check(-2, "dgp_num_placements")
        return int(n)

    def task_messages(self, offset: int, count: int) -> dict:
        """who_has / nbytes of the compute-task messages of placements [offset, offset +
        count) from the engine's state now (dgp_task_messages, _task_to_msg
        scheduler.py:3421-3450): ``dep_ptr`` [count + 1] / ``dep_task`` / ``dep_nbytes`` per
        dependency, ``holder_ptr`` [n_deps + 1] / ``holder_idx`` (ascending worker index)."""
        nd, nh = C.c_int64(0), C.c_int64(0)
        self._check(self.lib.dgp_task_messages(self.h, int(offset), int(count), C.byref(nd), C.byref(nh), None, None,
                                               None, None, None), "dgp_task_messages")
        out = dict(dep_ptr=np.zeros(count + 1, np.int64), dep_task=np.zeros(nd.value, np.int32),
                   dep_nbytes=np.zeros(nd.value, np.int64), holder_ptr=np.zeros(nd.value + 1, np.int64),
                   holder_idx=np.zeros(max(nh.value, 1), np.int32))
        self._check(self.lib.dgp_task_messages(self.h, int(offset), int(count), C.byref(nd), C.byref(nh),
                                               *(_ptr(out[k]) for k in ("dep_ptr", "dep_task", "dep_nbytes",
                                                                        "holder_ptr", "holder_idx"))),
                    "dgp_task_messages")
        out["holder_idx"] = out["holder_idx"][:nh.value]
        return out

    _PL_COLUMNS = (("pl_task", np.int32), ("pl_worker", np.int32), ("pl_comm", np.int64), ("pl_start", np.float64),
                   ("pl_wsnbytes", np.int64), ("pl_route", np.int8))

    def placements(self, offset: int = 0, count: int | None = None, columns=None) -> dict:
        """Placement-log entries [offset, offset + count); ``columns``: only those (the
        extension reads pl_task / pl_worker), one device round trip."""
        if count is None:
            count = self.num_placements() - offset
        out = {k: np.zeros(count, dt) for k, dt in self._PL_COLUMNS if columns is None or k in columns}
        self._check(self.lib.dgp_get_placements(self.h, offset, count, *[
            _ptr(out[k]) if k in out else None for k, _ in self._PL_COLUMNS]), "dgp_get_placements")
        return out

    def snapshots(self, max_rounds: int) -> dict:
        W = self.n_workers
        R = int(max_rounds)
        out = dict(round_nplaced=np.zeros(R, np.int32), round_occ=np.zeros((R, W)),
                   round_wnbytes=np.zeros((R, W), np.int64), round_nproc=np.zeros((R, W), np.int32),
                   round_idle=np.zeros((R, W), np.uint8), round_sat=np.zeros((R, W), np.uint8),
                   round_itc=np.zeros((R, W), np.uint8), round_nqueued=np.zeros(R, np.int32))
        n = C.c_int64(0)
        self._check(self.lib.dgp_get_snapshots(self.h, C.byref(n), *[_ptr(out[k]) for k in (
            "round_nplaced", "round_occ", "round_wnbytes", "round_nproc", "round_idle", "round_sat", "round_itc",
            "round_nqueued")]), "dgp_get_snapshots")
        return {k: v[:n.value] for k, v in out.items()}

    def task_states(self) -> np.ndarray:
        st = np.zeros(self.n_tasks, np.uint8)
        self._check(self.lib.dgp_get_task_states(self.h, _ptr(st)), "dgp_get_task_states")
        return st

    def set_timing(self, on: bool = True):
        self._check(self.lib.dgp_set_timing(self.h, 1 if on else 0), "dgp_set_timing")

    def stats(self) -> dict:
        out = np.zeros(49, np.int64)
        self._check(self.lib.dgp_stats(self.h, _ptr(out), 49), "dgp_stats")
        return dict(zip(("placements", "rounds", "dr_steps", "global_stimuli", "records", "walk_pos",
                         "cyc_setup", "cyc_local_steps", "cyc_global", "cyc_finish", "cyc_reserve", "cyc_max_step",
                         "cyc_exec_max", "cyc_exec_sum") + tuple(f"wave_phase{i}" for i in range(16))
                        + tuple(f"stall{i}" for i in range(8))
                        # resident service requests answered and the device's 100 MHz ticks spent
                        # answering / running / publishing them (summed)
                        + ("res_requests", "res_append_ticks", "res_run_ticks", "res_publish_ticks")
                        # when each role last finished a batch, after the request's append (summed)
                        + tuple(f"res_role_{r}_ticks" for r in ("bld", "pre", "reg", "claim", "exe", "seq", "wlk")),
                        map(int, out)))

    def kernel_times(self) -> dict:
        ms = np.zeros(8)
        n = np.zeros(8, np.int64)
        self._check(self.lib.dgp_kernel_times(self.h, _ptr(ms), _ptr(n), 8), "dgp_kernel_times")
        return {name: (float(ms[i]), int(n[i])) for i, name in enumerate(KERNEL_NAMES)}

    # ------------------------------------------------------------ WorkStealing
    def steal_balance(self, p: dict, group=None) -> dict:
        """steal_time_ratio for every processing task + one WorkStealing.balance()
        (distributed/stealing.py:241-277, :401-503) on the device.

        ``p``: nthreads, occ, nproc, wnbytes, idle, sat (per worker); total_occ,
        total_nthreads, bandwidth; victim, duration, fast, dep_ptr, dep_idx (per task);
        data_nbytes, data_get_nbytes and who_has as data_holder (one worker or -1) or
        holder_ptr / holder_idx (CSR); optionally task_prio / task_arrival (int64 per task):
        the tasks are then walked in ascending (priority, arrival) rather than input order
        (dgp_steal_order, sorted on the device). Returns levels, the ordered steal requests
        and the per-worker in-flight / idle / saturated state after the call.

        ``group``: a torch.distributed group of more than one rank (one engine per GPU,
        every rank passing the same ``p``): each rank computes its slice of the per-task
        thief rows and one all-gather gives every rank all of them (shard.py); the
        ordered walk then runs on every rank and gives the same result.
        """
        inputs, outputs, out, n, keep = self._steal_args(p)
        world = 1
        if group is not None:
            import torch.distributed as dist

            world = dist.get_world_size(group)
        if world == 1:
            self._check(self.lib.dgp_steal_balance(self.h, *inputs, *outputs), "dgp_steal_balance")
        else:
            self._steal_sharded(inputs, outputs, group)
        return self._steal_result(out, n)

    @staticmethod
    def _steal_result(out, n):
        k = int(n.value)
        for key in ("st_task", "st_victim", "st_thief", "st_level", "st_cost", "st_occ_victim", "st_occ_thief"):
            out[key] = out[key][:k]
        return out

    def _steal_args(self, p: dict):
        """ctypes arguments of dgp_steal_load / dgp_steal_balance (inputs) and of
        dgp_steal_run (outputs), the output arrays, the steal count and the kept buffers."""
        W = len(p["nthreads"])
        T = len(p["victim"])
        if "holder_ptr" in p:
            hptr, hidx = np.asarray(p["holder_ptr"], np.int64), np.asarray(p["holder_idx"], np.int32)
        else:
            h = np.asarray(p["data_holder"], np.int32)
            hptr = np.zeros(len(h) + 1, np.int64)
            hptr[1:] = np.cumsum(h >= 0)
            hidx = h[h >= 0].astype(np.int32)
        keep = []

        def a(x, dt):
            v = np.ascontiguousarray(x, dtype=dt)
            keep.append(v)
            return _ptr(v)

        out = dict(level=np.zeros(T, np.int8), st_task=np.zeros(T, np.int32), st_victim=np.zeros(T, np.int32),
                   st_thief=np.zeros(T, np.int32), st_level=np.zeros(T, np.int32), st_cost=np.zeros(T),
                   st_occ_victim=np.zeros(T), st_occ_thief=np.zeros(T), inflight_occ=np.zeros(W),
                   inflight_tasks=np.zeros(W, np.int32), idle_after=np.zeros(W, np.uint8),
                   sat_after=np.zeros(W, np.uint8), checked=np.zeros(W, np.uint8))
        n = C.c_int64(0)
        nd = len(p["data_nbytes"])
        inputs = (W, a(p["nthreads"], np.int32), a(p["occ"], np.float64), a(p["nproc"], np.int32),
                  a(p["wnbytes"], np.int64), a(p["idle"], np.uint8), a(p["sat"], np.uint8), float(p["total_occ"]),
                  int(p["total_nthreads"]), int(p["bandwidth"]), T, a(p["victim"], np.int32),
                  a(p["duration"], np.float64), a(p["fast"], np.uint8), a(p["dep_ptr"], np.int64),
                  a(p["dep_idx"], np.int32), nd, a(p["data_nbytes"], np.int64), a(p["data_get_nbytes"], np.int64),
                  a(hptr, np.int64), a(hidx, np.int32),
                  *((a(p["restr_ptr"], np.int64), a(p["restr_idx"], np.int32), a(p["restr_flags"], np.uint8))
                    if p.get("restr_flags") is not None else (None, None, None)),
                  a(p["level_in"], np.int8) if p.get("level_in") is not None else None,
                  a(p["inflight_occ_in"], np.float64) if p.get("inflight_occ_in") is not None else None,
                  a(p["inflight_tasks_in"], np.int32) if p.get("inflight_tasks_in") is not None else None)
        outputs = ([_ptr(out[k]) for k in ("level", "st_task", "st_victim", "st_thief", "st_level", "st_cost",
                                           "st_occ_victim", "st_occ_thief")] + [C.byref(n)]
                   + [_ptr(out[k]) for k in ("inflight_occ", "inflight_tasks", "idle_after", "sat_after", "checked")])
        if p.get("task_prio") is not None:  # rows in arrival slots: the device orders them (dgp_steal_order)
            self._check(self.lib.dgp_steal_order(self.h, T, a(p["task_prio"], np.int64), a(p["task_arrival"], np.int64)),
                        "dgp_steal_order")
        return inputs, outputs, out, n, keep

    def _steal_sharded(self, inputs, outputs, group):
        """dgp_steal_load -> this rank's thief rows -> all-gather of the rows (RCCL) ->
        dgp_steal_run (shard.py)."""
        import torch
        import torch.distributed as dist

        from .shard import chunk_rows, gather_rows, shard_range

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        ns = C.c_int64(0)
        self._check(self.lib.dgp_steal_load(self.h, *inputs, C.byref(ns)), "dgp_steal_load")
        n = int(ns.value)
        lo, hi = shard_range(n, rank, world)
        self._check(self.lib.dgp_steal_thief_rows(self.h, lo, hi), "dgp_steal_thief_rows")
        rb = int(self.lib.dgp_steal_row_bytes())
        # the engine's device; the zero-fill runs on torch's stream and the pack on the
        # engine's (a non-blocking stream): the fill must be done before the pack writes
        dev = torch.device("cuda", self.device)
        local = torch.zeros(max(chunk_rows(n, world), 0) * rb, dtype=torch.uint8, device=dev)
        torch.cuda.current_stream(dev).synchronize()
        if hi > lo:
            self._check(self.lib.dgp_steal_pack_rows(self.h, lo, hi, C.c_void_p(local.data_ptr())),
                        "dgp_steal_pack_rows")
        full = gather_rows(local, n, rb, group)
        torch.cuda.synchronize()  # the all-gather ran on torch's stream, the unpack runs on the engine's
        if n:
            self._check(self.lib.dgp_steal_unpack_rows(self.h, 0, n, C.c_void_p(full.data_ptr())),
                        "dgp_steal_unpack_rows")
        self._check(self.lib.dgp_steal_run(self.h, *outputs), "dgp_steal_run")
