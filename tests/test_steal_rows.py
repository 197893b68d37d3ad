"""GPUWorkStealing's incrementally kept task rows (distributed_amd/stealing.py StealRows)
against the full rebuild (steal_problem_from_state) on plain stand-ins of the reference's
objects (no dask needed): dependency rows longer than the slot row (KD), removals and slot
reuse, dependencies shared and dropped, unknown task durations (get_task_duration's
unknown_durations side effect), restrictions. The reference-plugin version of the same
check runs in tests/steal_ext_driver.py before every balance()."""
import numpy as np

from distributed_amd.stealing import StealRows, ordered_problem, steal_problem_from_state


class NS:  # a plain stand-in, hashed by identity like TaskState / WorkerState
    def __init__(self, **kw):
        self.__dict__.update(kw)


class Sched:
    def __init__(self, W, rng):
        self.workers = {f"tcp://w{i:03d}": NS(address=f"tcp://w{i:03d}", nthreads=2, occupancy=float(rng.random()),
                                              processing={}, nbytes=int(rng.integers(0, 1000)))
                        for i in range(W)}
        self.idle = {a: ws for a, ws in list(self.workers.items())[:3]}
        self.saturated = set(list(self.workers.values())[-2:])
        self.total_occupancy, self.total_nthreads, self.bandwidth = 12.5, 2 * W, 100_000_000
        self.unknown_durations = {}

    def get_task_duration(self, ts):  # scheduler.py:3024-3041
        d = ts.prefix.duration_average
        if d >= 0:
            return d
        self.unknown_durations.setdefault(ts.prefix.name, set()).add(ts)
        return 0.5

    def valid_workers(self, ts):
        return {self.workers[a] for a in ts.worker_restrictions}


def task(key, prio, deps, prefix, ws, restr=None):
    return NS(key=key, priority=prio, dependencies=deps, prefix=prefix, processing_on=ws, worker_restrictions=restr,
              host_restrictions=None, resource_restrictions=None, loose_restrictions=False)


def test_incremental_rows_equal_the_full_rebuild():
    rng = np.random.default_rng(7)
    s = Sched(16, rng)
    wss = list(s.workers.values())
    prefixes = [NS(name=f"p{j}", duration_average=-1.0 if j == 2 else 0.01 * (j + 1)) for j in range(4)]
    data = [NS(key=("d", i), nbytes=int(rng.integers(-1, 10_000)), who_has={wss[int(h)] for h in
                                                                          rng.choice(16, int(rng.integers(1, 3)),
                                                                                     replace=False)})
            for i in range(300)]
    for d in data:
        d.get_nbytes = (lambda d=d: d.nbytes if d.nbytes >= 0 else 1024)
    plugin = NS(scheduler=s, key_stealable={}, in_flight_occupancy={wss[1]: 0.25}, in_flight_tasks={wss[1]: 1})
    rows = StealRows()
    tasks = []
    for i in range(2000):
        k = int(rng.choice([0, 1, 2, 3, 9, 17]))  # rows past KD = 4 as well
        deps = [data[int(j)] for j in rng.choice(300, k, replace=False)]
        ws = wss[int(rng.integers(0, 16))]
        restr = {wss[int(rng.integers(0, 16))].address} if rng.random() < 0.05 else None
        ts = task(("t", i), (0, int(rng.integers(0, 50)), i), deps, prefixes[int(rng.integers(0, 4))], ws, restr)
        tasks.append(ts)

    def put(ts):
        level = int(rng.integers(1, 15))
        plugin.key_stealable[ts] = (ts.processing_on.address, level)
        rows.put(ts, ts.processing_on.address, level)

    def remove(ts):
        plugin.key_stealable.pop(ts, None)
        rows.remove(ts)

    def check():
        a, ta, _ = steal_problem_from_state(plugin)
        b, slots, _ = rows.problem(plugin)
        b, slots = ordered_problem(b, slots)  # the device's walk order
        tb = [rows.task[int(i)] for i in slots]
        assert ta == tb
        assert set(a) == set(b)
        for k in a:
            if k in ("dep_idx", "data_nbytes", "data_get_nbytes", "holder_ptr", "holder_idx"):
                continue
            if isinstance(a[k], np.ndarray):
                assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), k
            else:
                assert a[k] == b[k], k

        def per_task(p):
            out = []
            for t in range(len(p["dep_ptr"]) - 1):
                r = p["dep_idx"][p["dep_ptr"][t]:p["dep_ptr"][t + 1]]
                assert np.all(np.diff(r) > 0)
                out.append(sorted((int(p["data_nbytes"][d]), int(p["data_get_nbytes"][d]),
                                   tuple(p["holder_idx"][p["holder_ptr"][d]:p["holder_ptr"][d + 1]])) for d in r))
            return out

        assert per_task(a) == per_task(b)

    for ts in tasks[:1500]:
        put(ts)
    check()
    for ts in tasks[::3]:  # removals (free slots, dependencies dropped), then reuse
        remove(ts)
    check()
    for ts in tasks[1500:]:
        put(ts)
    for ts in tasks[1:1500:7]:  # a task put again (a recalculated cost) moves to the end of its ties
        put(ts)
    check()
    # who_has changes through the scheduler's replica hooks (add_replica / remove_replica /
    # remove_all_replicas), which the plugin forwards to the rows
    for i, d in enumerate(data[:60]):
        ws = wss[(i * 5) % 16]
        if i % 3 == 0 and len(d.who_has) > 1:
            h = sorted(d.who_has, key=lambda w: w.address)[0]
            d.who_has.discard(h)
            rows.replica(d, h.address, -1)
        elif i % 3 == 1:
            d.who_has.add(ws)
            rows.replica(d, ws.address, +1)
        else:
            for w in wss[:12]:  # more holders than a dependency row keeps inline
                d.who_has.add(w)
                rows.replica(d, w.address, +1)
    check()
    for d in data[60:70]:
        for w in list(d.who_has):
            d.who_has.discard(w)
        rows.replicas_cleared(d)
    check()
    assert "p2" in s.unknown_durations
    rows.clear()
    assert len(rows) == 0
