"""Times the REFERENCE's own Python placement path (build container only: python3.9 +
/root/reference through tests/golden/_refshim.py; the reference never travels to the GPU
box). One process, one core (the scheduler is single-threaded), PYTHONHASHSEED=0.

    PYTHONHASHSEED=0 taskset -c 2 /opt/conda/bin/python3.9 tools/ref_python_time.py c2|c3|c4|c4mtr [--out FILE]

c2 / c3: the BASELINE.json C2 (1M-task random DAG x 1,024 workers, saturation 1.1) and
C3 (P2P-shuffle shape, 66,666 partitions x 512 workers) graphs of distributed_amd/graphs.py,
replayed exactly as tests/golden/gen_golden.py does (update_graph's recommendations, then
every round's task-finished stimuli through _transition + _transitions +
stimulus_queue_slots_maybe_opened), on the reference SchedulerState with no
instrumentation in the decisions (plain sets, no recording subclass). Reported:
placement-only time = the time spent inside the three -> processing transition functions
of the reference's own _TRANSITIONS_TABLE (scheduler.py:2889-2912:
_transition_waiting_processing :2313, _transition_queued_processing :2797,
_transition_no_worker_processing :2121), and the whole replay's time.
c4: one reference WorkStealing.balance() (stealing.py:401-503) on the C4 scenario of
tests/golden/gen_steal.py at 100k stealable tasks x 4,096 workers (as SURVEY §6)."""
from __future__ import annotations

import json
import operator
import os
import platform
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
if os.environ.get("PYTHONHASHSEED") != "0":
    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, PYTHONHASHSEED="0")))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import warnings  # noqa: E402

warnings.filterwarnings("ignore")
import _refshim  # noqa: E402

_refshim.install()
import dask  # noqa: E402
import numpy as np  # noqa: E402

import distributed.scheduler  # noqa: E402,F401
import gen_golden as GG  # noqa: E402


def timed_table(cls, acc):
    """The reference table with its three -> processing entries wrapped by a timer."""
    table = dict(cls._TRANSITIONS_TABLE)
    for k in (("waiting", "processing"), ("queued", "processing"), ("no-worker", "processing")):
        f = table[k]

        def wrap(self, key, stimulus_id, _f=f, **kw):
            a = time.perf_counter()
            try:
                return _f(self, key, stimulus_id, **kw)
            finally:
                acc[0] += time.perf_counter() - a
                acc[1] += 1
        table[k] = wrap
    return table


def placement_run(g, cfg):
    from sortedcontainers import SortedDict

    from distributed.collections import HeapSet
    from distributed.core import Status
    from distributed.scheduler import ClientState, Scheduler, SchedulerState, WorkerState

    acc = [0.0, 0]
    placed = []

    class S(SchedulerState):
        def transitions(self, recommendations, stimulus_id):
            self._transitions(recommendations, {}, {}, stimulus_id)

        stimulus_queue_slots_maybe_opened = Scheduler.stimulus_queue_slots_maybe_opened

        def log_event(self, *args, **kwargs):
            pass

    S._TRANSITIONS_TABLE = timed_table(SchedulerState, acc)
    orig_add = SchedulerState._add_to_processing

    def _add_to_processing(self, ts, ws, stimulus_id):  # the replay needs the round's placements
        placed.append(ts)
        return orig_add(self, ts, ws, stimulus_id)

    S._add_to_processing = _add_to_processing
    t_build = time.perf_counter()
    s = S(aliases={}, clients={}, workers=SortedDict(), host_info={}, resources={}, tasks={}, unrunnable=set(),
          queued=HeapSet(key=operator.attrgetter("priority")), validate=False, plugins=())
    W = len(g["nthreads"])
    for i in range(W):
        addr = f"tcp://w{i:05d}:1"
        ws = WorkerState(address=addr, status=Status.running, pid=0, name=addr, nthreads=int(g["nthreads"][i]),
                         memory_limit=0, local_directory="", nanny=None, server_id=addr, scheduler=s)
        s.workers[addr] = ws
        s.running.add(ws)
        s.aliases[addr] = addr
        s.total_nthreads += ws.nthreads
        s.check_idle_saturated(ws)
    keys = g["keys"] or GG.make_keys(g)
    cs = ClientState("client-0")
    s.clients["client-0"] = cs
    run_spec = (operator.add, (), {})
    tss = []
    for t, key in enumerate(keys):
        ts = s.new_task(key, run_spec, "released")
        ts.priority = (0, 1, int(g["prio"][t]))
        ov = int(g["rootish_override"][t])
        if ov >= 0:
            ts._rootish = bool(ov)
        tss.append(ts)
    ptr, idx = g["dep_ptr"], g["dep_idx"]
    for t, ts in enumerate(tss):
        for d in idx[ptr[t]:ptr[t + 1]]:
            ts.add_dependency(tss[int(d)])
    for t, ts in enumerate(tss):
        if g["wanted"][t]:
            ts.who_wants = {cs}
            cs.wants_what.add(ts)
    index = {ts.key: i for i, ts in enumerate(tss)}
    t_build = time.perf_counter() - t_build
    t0 = time.perf_counter()
    recs = {}
    for ts in sorted(tss, key=operator.attrgetter("priority"), reverse=True):
        recs[ts.key] = "waiting"
    s._transitions(recs, {}, {}, "update-graph")
    done, rounds = 0, 0
    while True:
        cur = len(placed)
        batch = placed[done:cur]
        done = cur
        if not batch:
            break
        rounds += 1
        for ts in batch:
            i = index[ts.key]
            sid = f"task-finished-{i}"
            r, cm, wm = s._transition(ts.key, "memory", sid, worker=ts.processing_on.address,
                                      nbytes=int(g["nbytes"][i]), type=None, typename="int",
                                      startstops=[{"action": "compute", "start": float(g["start"][i]),
                                                   "stop": float(g["stop"][i])}])
            s._transitions(r, cm, wm, sid)
            s.stimulus_queue_slots_maybe_opened(stimulus_id=sid)
    total = time.perf_counter() - t0
    return dict(placements=len(placed), processing_calls=acc[1], placement_only_s=acc[0],
                placement_only_per_s=acc[1] / acc[0], replay_s=total, replay_per_s=len(placed) / total,
                rounds=rounds, state_build_s=t_build)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    cfg = GG.config_dict(1.1)
    if which == "c2":
        g = GG.graphs.random_dag(1_000_000, 1024, seed=0)
        res = dict(config="C2: random_dag(1_000_000, 1024, seed=0), saturation 1.1", **placement_run(g, cfg))
    elif which == "c3":
        g = GG.graphs.shuffle_graph(66_666, 512)
        res = dict(config="C3: shuffle_graph(66_666, 512), saturation 1.1", **placement_run(g, cfg))
    elif which == "c4":
        import gen_steal as GS

        T = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 100_000
        a = time.perf_counter()
        s, steal, widx, tidx, data, work, deps_of, events, comms = GS.build(4096, T, 2, 0.1, 1)
        built = time.perf_counter() - a
        a = time.perf_counter()
        steal.balance()
        secs = time.perf_counter() - a
        n_req = sum(len(c.sent) for c in comms.values())
        res = dict(config=f"C4: gen_steal.build(4096 workers, {T} tasks, nthreads 2, hot 10%, seed 1)",
                   balance_s=secs, steal_requests=n_req, state_build_s=built,
                   move_task_request_note="included: the reference's balance() sends each request itself")
    elif which == "c4mtr":  # the reference's own WorkStealing.move_task_request, per request
        import gen_steal as GS

        T = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 100_000
        s, steal, widx, tidx, data, work, deps_of, events, comms = GS.build(4096, T, 2, 0.1, 1)
        tasks = sorted(steal.key_stealable, key=lambda ts: ts.priority)
        thieves = sorted(s.idle.values(), key=lambda ws: ws.address)
        n = min(20_000, len(tasks))
        a = time.perf_counter()
        for i, ts in enumerate(tasks[:n]):
            steal.move_task_request(ts, ts.processing_on, thieves[i % len(thieves)])
        secs = time.perf_counter() - a
        res = dict(config=f"C4: gen_steal.build(4096 workers, {T} tasks, nthreads 2, hot 10%, seed 1); "
                          f"move_task_request for the first {n} stealable tasks (priority order), thieves round-robin",
                   move_task_request_us=round(1e6 * secs / n, 2), requests=n)
    else:
        raise SystemExit(f"unknown config {which}")
    res.update(reference="/root/reference (fjetter/distributed) SchedulerState / WorkStealing, unmodified, via "
                         "tests/golden/_refshim.py", python=sys.version.split()[0], dask=dask.__version__,
               cores=1, hashseed=0, host=platform.processor() or platform.machine(),
               cpu_affinity=sorted(os.sched_getaffinity(0)), script="tools/ref_python_time.py")
    print(json.dumps(res, indent=1), flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
