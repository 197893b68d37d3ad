"""Seams of the drop-in extension (distributed_amd/ext.py) that need no reference scheduler:
a stand-in SchedulerState / WorkStealing pair with the attributes the extension wraps.

A stimulus the scheduler decided itself leaves the engine suspended until its resync; a
steal confirmation (stealing.py:333-399) or a balance() call (:401-503) that comes next is a
stimulus of its own, so the resync runs before the engine is asked to move a task or to take
idle / saturated changes (the engine refuses both while a resync is pending).
"""
import asyncio
from types import SimpleNamespace

from distributed_amd.ext import GPUPlacementExtension


class _Steal:
    def __init__(self, sched):
        self.sched = sched

    async def move_task_confirm(self, *, key, state, stimulus_id, worker=None):
        ts = self.sched.tasks[key]  # confirm: the task moves to the thief
        ts.processing_on = self.sched.workers[worker]

    def balance(self):
        self.sched.idle = {"b": self.sched.workers["b"]}  # the thief is idle afterwards


class _Sched:
    _TRANSITIONS_TABLE = {("waiting", "processing"): lambda *a, **k: None,
                          ("queued", "processing"): lambda *a, **k: None}

    def __init__(self):
        self.workers = {a: SimpleNamespace(address=a) for a in ("a", "b")}
        self.tasks = {"x": SimpleNamespace(key="x", state="processing", processing_on=self.workers["a"])}
        self.idle, self.saturated, self.plugins = {}, set(), {}
        self.extensions = {"stealing": _Steal(self)}

    def _add_to_processing(self, ts, ws, stimulus_id):
        return None

    def add_replica(self, ts, ws):
        return None

    def remove_replica(self, ts, ws):
        return None


class _Engine:
    def __init__(self, calls):
        self.calls = calls

    def move_task(self, t, w):
        self.calls.append(("move_task", t, w))

    def set_worker_flags(self, workers, idle, saturated):
        self.calls.append(("set_worker_flags", list(workers), list(idle), list(saturated)))

    def num_placements(self):
        return 0


def _suspended_extension(calls):
    s = _Sched()
    ext = GPUPlacementExtension(s)
    ext.engine = _Engine(calls)
    ext.task_index, ext.keys = {"x": 0}, ["x"]
    ext.worker_index, ext.workers = {"a": 0, "b": 1}, ["a", "b"]

    def resync():
        calls.append("resync")
        ext.suspended = False

    ext._resync = resync
    ext.suspended = True
    return s, ext


def test_steal_confirmation_resyncs_first():
    calls = []
    s, ext = _suspended_extension(calls)
    asyncio.run(s.extensions["stealing"].move_task_confirm(key="x", state="processing", stimulus_id="s", worker="b"))
    assert calls == ["resync", ("move_task", 0, 1)]
    assert ext.active


def test_balance_resyncs_first():
    calls = []
    s, ext = _suspended_extension(calls)
    s.extensions["stealing"].balance()
    assert calls == ["resync", ("set_worker_flags", [1], [1], [0])]
    assert ext.active
