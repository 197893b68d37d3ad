"""Synthetic task graphs for the placement hot path (BASELINE.json configs C2/C3/C5).

numpy-only on purpose: this module is also loaded by path from the golden-vector
generator (``tests/golden/gen_golden.py``), which runs the *reference* scheduler
under the image's python3.9 — so it must not import torch or the HIP library.

A graph is a plain ``dict`` of numpy arrays ("graph dict"):

=====================  ==========  =================================================
field                  dtype       meaning (reference attribute it mirrors)
=====================  ==========  =================================================
``dep_ptr/dep_idx``    i64 / i32   CSR of ``TaskState.dependencies`` (deduplicated;
                                   ``distributed/scheduler.py:1219``)
``prio``               i64         rank of ``TaskState.priority`` (0 = runs first;
                                   only the order of the tuples matters, :1207)
``prefix_id``          i32         ``TaskState.prefix`` (``key_split``, :1829)
``group_id``           i32         ``TaskState.group`` (``key_split_group``, :1835)
``wanted``             u8          ``bool(TaskState.who_wants)`` (client futures)
``rootish_override``   i8          ``TaskState._rootish`` (-1 = None, :2940)
``nbytes``             i64         ``nbytes`` the worker reports on completion
``start/stop``         f64         the task's ``startstops`` compute interval
``nthreads``           i32[W]      ``WorkerState.nthreads`` of the simulated workers
``prefix_names``       list[str]   TaskPrefix names (index = prefix id)
``group_names``        list[str]   TaskGroup names (index = group id)
``group_prefix``       i32[G]      ``TaskGroup.prefix``
``prefix_default_dur`` f64[P]      ``default-task-durations`` entry or -1 (:964-968)
``keys``               list|None   reference task keys (golden fixtures only)
=====================  ==========  =================================================
"""
from __future__ import annotations

import numpy as np

# a hex token that key_split() drops (it contains digits), like dask's tokenize()
TOKEN = "0a1b2c3d4e5f60718293a4b5c6d7e8f9"


def _csr_from_rows(rows):
    ptr = np.zeros(len(rows) + 1, dtype=np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    idx = np.concatenate([np.asarray(r, dtype=np.int32) for r in rows]) if rows else np.zeros(0, np.int32)
    return ptr, idx.astype(np.int32)


def _dedup_rows_sorted(draws: np.ndarray):
    """Per-row ``numpy.unique`` of a 2-D int array, returned as CSR."""
    s = np.sort(draws, axis=1)
    keep = np.ones_like(s, dtype=bool)
    keep[:, 1:] = s[:, 1:] != s[:, :-1]
    counts = keep.sum(axis=1)
    return s[keep], counts


def _finish(g: dict) -> dict:
    n = len(g["prio"])
    deg_out = np.bincount(g["dep_idx"], minlength=n) if len(g["dep_idx"]) else np.zeros(n, np.int64)
    if "wanted" not in g:
        # sinks are what the client holds futures for (Client.compute of the collection)
        g["wanted"] = (deg_out == 0).astype(np.uint8)
    g.setdefault("rootish_override", np.full(n, -1, np.int8))
    g.setdefault("keys", None)
    g["n_tasks"] = n
    for k, dt in (("dep_ptr", np.int64), ("dep_idx", np.int32), ("prio", np.int64),
                  ("prefix_id", np.int32), ("group_id", np.int32), ("wanted", np.uint8),
                  ("rootish_override", np.int8), ("nbytes", np.int64), ("start", np.float64),
                  ("stop", np.float64), ("nthreads", np.int32), ("group_prefix", np.int32),
                  ("prefix_default_dur", np.float64)):
        g[k] = np.ascontiguousarray(g[k], dtype=dt)
    return g


def random_dag(n_tasks: int, n_workers: int, *, seed: int = 0, fanin: int = 4,
               root_frac: float = 0.1, window_mult: int = 4, n_inner_prefixes: int = 1,
               random_durations: bool = False, nthreads: int | str = 1) -> dict:
    """Config C2: random DAG, roots = N/10, every other task i draws
    ``unique(rng.integers(max(0, i - 4W), i, 4))`` dependencies, output nbytes
    ``int(lognormal(10, 2))``, priority ``(0, 1, i)``, compute interval [0.0, 0.01].

    Variants used by the parity fixtures: several inner prefixes (exercises the
    insertion-ordered occupancy sum of ``_calc_occupancy`` :1889-1900), random task
    durations (exercises the ``TaskPrefix.add_duration`` EWMA :977-985) and
    heterogeneous ``nthreads``.
    """
    rng = np.random.default_rng(seed)
    n = int(n_tasks)
    r = max(1, int(n * root_frac))
    nbytes = rng.lognormal(10, 2, n).astype(np.int64)
    i = np.arange(r, n, dtype=np.int64)
    lo = np.maximum(0, i - window_mult * n_workers)
    draws = rng.integers(lo[:, None], i[:, None], size=(n - r, fanin))
    flat, counts = _dedup_rows_sorted(draws)
    dep_ptr = np.zeros(n + 1, np.int64)
    dep_ptr[r + 1:] = np.cumsum(counts)
    stop = np.full(n, 0.01)
    if random_durations:
        stop = rng.uniform(0.001, 0.1, n)
    if nthreads == "random":
        nth = rng.integers(1, 5, n_workers)
    else:
        nth = np.full(n_workers, int(nthreads))
    k = int(n_inner_prefixes)
    prefix_names = ["root"] + (["inner"] if k == 1 else [f"inner{j}" for j in range(k)])
    prefix_id = np.zeros(n, np.int32)
    prefix_id[r:] = 1 + (np.arange(r, n) % k)
    group_names = [f"{p}-{TOKEN}" for p in prefix_names]
    return _finish(dict(
        name=f"random_dag_{n}x{n_workers}", dep_ptr=dep_ptr, dep_idx=flat.astype(np.int32),
        prio=np.arange(n, dtype=np.int64), prefix_id=prefix_id, group_id=prefix_id.copy(),
        prefix_names=prefix_names, group_names=group_names,
        group_prefix=np.arange(len(prefix_names)), prefix_default_dur=np.full(len(prefix_names), -1.0),
        nbytes=nbytes, start=np.zeros(n), stop=stop, nthreads=nth))


def restrict(g: dict, frac: float, *, seed: int = 0, max_valid: int = 8, empty_frac: float = 0.1,
             loose_frac: float = 0.5) -> dict:
    """Worker restrictions on a fraction of the tasks (``TaskState.worker_restrictions`` /
    ``loose_restrictions``, scheduler.py:1338-1354, :4908-4922), already resolved to the
    valid worker indices of ``valid_workers`` (:3043-3107) as CSR ``restr_ptr`` /
    ``restr_idx`` (ascending). ``restr_flags`` bit 0: the task is restricted; bit 1: loose.
    A restricted task whose valid set is empty (its restriction names no worker of the
    cluster) goes to ``no-worker`` unless loose (decide_worker :8584-8586)."""
    rng = np.random.default_rng(seed)
    n, W = g["n_tasks"], len(g["nthreads"])
    flags = np.zeros(n, np.uint8)
    rows = [[] for _ in range(n)]
    for t in np.flatnonzero(rng.random(n) < frac):
        flags[t] = 1 | (2 if rng.random() < loose_frac else 0)
        if rng.random() >= empty_frac:
            k = int(rng.integers(1, max_valid + 1))
            rows[t] = sorted(set(rng.integers(0, W, k).tolist()))
    ptr, idx = _csr_from_rows(rows)
    g = dict(g)
    g.update(restr_ptr=ptr, restr_idx=idx, restr_flags=flags)
    return g


def star(n_leaves: int, n_workers: int) -> dict:
    """One root and ``n_leaves`` non-rootish leaves that depend on it: the root's completion
    places every leaf on the root's worker (its only candidate, scheduler.py:8550-8593),
    and the next round completes them one after another, each touching that one worker.
    The slope of replay time over ``n_leaves`` is the engine's link latency within a round,
    the constant of bench.py's latency bound (C3's unpack phase has the same shape)."""
    n = int(n_leaves) + 1
    dep_ptr = np.zeros(n + 1, np.int64)
    dep_ptr[2:] = np.arange(1, n)
    prefix_id = np.minimum(np.arange(n), 1).astype(np.int32)
    return _finish(dict(
        name=f"star_{n_leaves}x{n_workers}", dep_ptr=dep_ptr, dep_idx=np.zeros(n - 1, np.int32),
        prio=np.arange(n, dtype=np.int64), prefix_id=prefix_id, group_id=prefix_id.copy(),
        prefix_names=["hub", "leaf"], group_names=[f"hub-{TOKEN}", f"leaf-{TOKEN}"],
        group_prefix=np.arange(2), prefix_default_dur=np.full(2, -1.0),
        rootish_override=np.zeros(n, np.int8), nbytes=np.full(n, 1000, np.int64), start=np.zeros(n),
        stop=np.full(n, 0.01), nthreads=np.ones(n_workers)))


def shuffle_graph(n_partitions: int, n_workers: int, *, seed: int = 2, restricted: bool = False,
                  live: bool = False) -> dict:
    """Config C3: the P2P-shuffle graph shape of ``distributed/shuffle/_shuffle.py:276-306``:
    P inputs -> P ``shuffle-transfer`` -> one ``shuffle-barrier`` (fan-in P) -> P
    ``shuffle-p2p`` unpack tasks, the unpacks forced non-rootish
    (``_ensure_output_tasks_are_non_rootish``, ``_scheduler_plugin.py:254-278``).
    Transfer outputs are ``int(lognormal(6, 1))`` bytes. Priorities follow a
    depth-first order: input i, transfer i, ..., barrier, unpack 0..P-1.

    ``restricted``: each unpack task pinned to its output partition's worker, as the
    shuffle plugin does at the barrier (``restrict_task`` / ``_set_restriction``,
    ``_scheduler_plugin.py:101-115``, worker ``_get_worker_for_range_sharding``
    ``_shuffle.py:612-617``: index ``W * i // P``): decide_worker's candidates (the
    barrier's holder) miss the valid set, so each unpack goes to its pinned worker.

    ``live``: the graph as the client submits it, before the shuffle runs: the unpacks'
    ``_rootish`` is still None (the plugin sets it False when the first transfer starts,
    the live lifecycle of tests/golden/gen_service.py ``p2p``).
    """
    rng = np.random.default_rng(seed)
    p = int(n_partitions)
    n = 3 * p + 1
    inp = np.arange(p)
    tr = p + np.arange(p)
    bar = 2 * p
    unp = 2 * p + 1 + np.arange(p)
    rows = [[] for _ in range(n)]
    for j in range(p):
        rows[tr[j]] = [inp[j]]
        rows[unp[j]] = [bar]
    rows[bar] = list(tr)
    dep_ptr, dep_idx = _csr_from_rows(rows)
    prio = np.zeros(n, np.int64)
    prio[inp] = 2 * np.arange(p)
    prio[tr] = 2 * np.arange(p) + 1
    prio[bar] = 2 * p
    prio[unp] = 2 * p + 1 + np.arange(p)
    nbytes = np.zeros(n, np.int64)
    nbytes[inp] = rng.lognormal(10, 1, p).astype(np.int64)
    nbytes[tr] = rng.lognormal(6, 1, p).astype(np.int64)
    nbytes[bar] = 0
    nbytes[unp] = rng.lognormal(10, 1, p).astype(np.int64)
    prefix_names = ["input", "shuffle-transfer", "shuffle-barrier", "shuffle"]
    prefix_id = np.zeros(n, np.int32)
    prefix_id[tr] = 1
    prefix_id[bar] = 2
    prefix_id[unp] = 3
    rootish = np.full(n, -1, np.int8)
    if not live:
        rootish[unp] = 0
    group_names = [f"input-{TOKEN}", f"shuffle-transfer-{TOKEN}", "shuffle-barrier", f"shuffle-p2p-{TOKEN}"]
    extra = {}
    if restricted:
        rrows = [[] for _ in range(n)]
        for j in range(p):
            rrows[unp[j]] = [int(n_workers) * j // p]
        rptr, ridx = _csr_from_rows(rrows)
        rflags = np.zeros(n, np.uint8)
        rflags[unp] = 1
        extra = dict(restr_ptr=rptr, restr_idx=ridx, restr_flags=rflags)
    return _finish(dict(**extra,
        name=f"shuffle_{p}x{n_workers}" + ("_restricted" if restricted else "") + ("_live" if live else ""),
        dep_ptr=dep_ptr, dep_idx=dep_idx,
        prio=prio,
        prefix_id=prefix_id, group_id=prefix_id.copy(), prefix_names=prefix_names,
        group_names=group_names, group_prefix=np.arange(4), prefix_default_dur=np.full(4, -1.0),
        rootish_override=rootish, nbytes=nbytes, start=np.zeros(n), stop=np.full(n, 0.01),
        nthreads=np.ones(n_workers, np.int32)))


def map_tree_reduce(n_map: int, n_workers: int, *, fanin: int = 8, seed: int = 3) -> dict:
    """Config C5: ``n_map`` map tasks reduced by a ``fanin``-ary tree. Output nbytes
    ``int(lognormal(10, 2))``. Priorities are the depth-first post-order that
    ``dask.order`` gives a tree reduction (each reduce node right after its inputs).
    Task index order = map tasks first, then each reduce level.
    """
    rng = np.random.default_rng(seed)
    m = int(n_map)
    levels = [m]
    while levels[-1] > 1:
        levels.append((levels[-1] + fanin - 1) // fanin)
    offs = np.cumsum([0] + levels)
    n = int(offs[-1])
    dep_ptr = np.zeros(n + 1, np.int64)
    dep_chunks = []
    ptr = 0
    for lv in range(1, len(levels)):
        cnt = levels[lv]
        child_n = levels[lv - 1]
        k = np.arange(cnt)
        lo = k * fanin
        hi = np.minimum(lo + fanin, child_n)
        sizes = hi - lo
        dep_ptr[offs[lv] + 1: offs[lv] + cnt + 1] = ptr + np.cumsum(sizes)
        ptr += int(sizes.sum())
        starts = np.repeat(lo, sizes)
        within = np.arange(int(sizes.sum())) - np.repeat(np.cumsum(sizes) - sizes, sizes)
        dep_chunks.append(offs[lv - 1] + starts + within)
    # map tasks have no deps: dep_ptr[1..m] = 0 already; make it monotone
    dep_ptr = np.maximum.accumulate(dep_ptr)
    dep_idx = np.concatenate(dep_chunks).astype(np.int32) if dep_chunks else np.zeros(0, np.int32)
    # depth-first post-order priority (iterative, vectorised per level):
    # rank of a node = position in post-order traversal of the tree
    prio = np.zeros(n, np.int64)
    # subtree sizes per level, bottom up
    sub = [np.ones(levels[0], np.int64)]
    for lv in range(1, len(levels)):
        child = sub[-1]
        cnt = levels[lv]
        s = np.add.reduceat(child, np.arange(cnt) * fanin) + 1
        sub.append(s)
    # first rank in each subtree, top down
    first = [None] * len(levels)
    first[-1] = np.zeros(1, np.int64)
    for lv in range(len(levels) - 1, 0, -1):
        child = sub[lv - 1]
        f = first[lv]
        cnt_child = levels[lv - 1]
        parent = np.arange(cnt_child) // fanin
        # offset of child inside its parent's subtree = sum of earlier siblings' sizes
        csum = np.cumsum(child) - child
        base = csum - csum[(parent * fanin)]
        first[lv - 1] = f[parent] + base
    for lv in range(len(levels)):
        prio[offs[lv]:offs[lv + 1]] = first[lv] + sub[lv] - 1
    nbytes = rng.lognormal(10, 2, n).astype(np.int64)
    prefix_names = ["map", "reduce"]
    prefix_id = np.ones(n, np.int32)
    prefix_id[:m] = 0
    group_id = np.zeros(n, np.int32)
    for lv in range(1, len(levels)):
        group_id[offs[lv]:offs[lv + 1]] = lv
    group_names = [f"map-{TOKEN}"] + [f"reduce-l{lv}-{TOKEN}" for lv in range(1, len(levels))]
    group_prefix = np.array([0] + [1] * (len(levels) - 1))
    return _finish(dict(
        name=f"map_tree_reduce_{m}x{n_workers}", dep_ptr=dep_ptr, dep_idx=dep_idx, prio=prio,
        prefix_id=prefix_id, group_id=group_id, prefix_names=prefix_names,
        group_names=group_names, group_prefix=group_prefix, prefix_default_dur=np.full(2, -1.0),
        nbytes=nbytes, start=np.zeros(n), stop=np.full(n, 0.01),
        nthreads=np.ones(n_workers, np.int32)))


PLACEMENT_KEYS = ("pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")


def placement_digest(out: dict) -> str:
    """sha256 over a placement log's six arrays (task, worker, comm bytes, fp64 start
    bits, ws.nbytes, route), in log order: pins full-size replays whose oracle run is
    too slow for a test (tests/golden/c5_full_digest.json)."""
    import hashlib

    h = hashlib.sha256()
    for k in PLACEMENT_KEYS:
        h.update(np.ascontiguousarray(out[k]).tobytes())
    return h.hexdigest()


def check_graph(g: dict) -> None:
    """Structural invariants the engine relies on (raise ValueError otherwise)."""
    n = g["n_tasks"]
    if g["dep_ptr"][0] != 0 or g["dep_ptr"][-1] != len(g["dep_idx"]) or np.any(np.diff(g["dep_ptr"]) < 0):
        raise ValueError("bad dep_ptr")
    if len(g["dep_idx"]) and (g["dep_idx"].min() < 0 or g["dep_idx"].max() >= n):
        raise ValueError("dep_idx out of range")
    if len(np.unique(g["prio"])) != n:
        raise ValueError("priorities must be unique")
    src = np.repeat(np.arange(n), np.diff(g["dep_ptr"]))
    if np.any(g["prio"][g["dep_idx"]] >= g["prio"][src]):
        # dask.order priorities are topological; the transition engine's LIFO
        # order (SURVEY §8a checklist 1) relies on it
        raise ValueError("priorities are not topological")
    for k in ("prefix_id", "group_id", "wanted", "rootish_override", "nbytes", "start", "stop"):
        if len(g[k]) != n:
            raise ValueError(f"{k} has wrong length")


def steal_problem(n_workers: int, n_tasks: int, *, nthreads: int = 2, hot_frac: float = 0.1, seed: int = 1,
                  n_prefixes: int = 8, zipf_a: float = 1.5, replicas: int = 1, occ_quantum: float = 0.0,
                  restrict: float = 0.0) -> dict:
    """A WorkStealing.balance() input in the shape of BASELINE.json's C4:
    D = T/4 memory-resident dependencies (``int(lognormal(16, 3))`` bytes) on uniform
    workers; T processing tasks with 1-2 of them (5 % dependency-free -> level 0) in
    prefixes with durations 10 ms * 2^j, on the ``hot_frac`` "hot" workers chosen
    ``zipf(a) mod |hot|``. Occupancy = the tasks' durations + the bytes of their remote
    dependencies / bandwidth (each dependency once per worker); idle / saturated follow
    ``check_idle_saturated`` (scheduler.py:2949-2995). The arrays of
    ``PlacementEngine.steal_balance`` / ``oracle.steal_balance``.

    ``replicas`` > 1 gives every dependency 1..replicas distinct holders (who_has as
    holder_ptr / holder_idx); ``occ_quantum`` > 0 rounds occupancies to that grid, so many
    thieves tie on stack time."""
    rng = np.random.default_rng(seed)
    W, T = int(n_workers), int(n_tasks)
    bw = 100_000_000
    D = max(T // 4, 1)
    hot = rng.choice(W, size=max(int(round(W * hot_frac)), 1), replace=False)
    holder = rng.integers(0, W, D).astype(np.int32)
    nbytes = rng.lognormal(16, 3, D).astype(np.int64)
    pid = rng.integers(0, n_prefixes, T)
    duration = (0.01 * 2.0 ** pid).astype(np.float64)
    k = np.where(rng.random(T) < 0.05, 0, rng.integers(1, 3, T))
    deps = [np.unique(rng.integers(0, D, kk)) for kk in k]
    dep_ptr = np.zeros(T + 1, np.int64)
    dep_ptr[1:] = np.cumsum([len(d) for d in deps])
    dep_idx = np.concatenate(deps).astype(np.int32) if T else np.zeros(0, np.int32)
    victim = hot[rng.zipf(zipf_a, T) % len(hot)].astype(np.int32)
    nth = np.full(W, nthreads, np.int32)
    nproc = np.bincount(victim, minlength=W).astype(np.int32)
    occ = np.zeros(W)
    np.add.at(occ, victim, duration)
    if replicas > 1:
        extra = [rng.choice(W, size=int(rng.integers(0, replicas)), replace=False) for _ in range(D)]
        hs = [np.unique(np.concatenate([[holder[d]], extra[d]])).astype(np.int32) for d in range(D)]
    else:
        hs = [holder[d:d + 1] for d in range(D)]
    need = {}
    for t in range(T):
        for d in deps[t]:
            if victim[t] not in hs[d]:
                need.setdefault(int(victim[t]), set()).add(int(d))
    netocc = np.zeros(W, np.int64)
    for w, ds in need.items():
        netocc[w] = int(nbytes[list(ds)].sum())
    occ = occ + netocc / bw
    if occ_quantum > 0:
        occ = np.round(occ / occ_quantum) * occ_quantum
    hptr = np.zeros(D + 1, np.int64)
    hptr[1:] = np.cumsum([len(h) for h in hs])
    hidx = np.concatenate(hs).astype(np.int32)
    wnbytes = np.bincount(hidx, weights=np.repeat(nbytes, np.diff(hptr)), minlength=W).astype(np.int64)
    total_occ = float(occ.sum())
    tn = int(nth.sum())
    avg = total_occ / tn
    idle = ((nproc < nth) | (occ < nth * avg / 2)).astype(np.uint8)
    pend = np.where(nproc > nth, occ * (nproc - nth) / np.maximum(nproc * nth, 1), 0.0)
    sat = ((idle == 0) & (nproc > nth) & (pend > 0.4) & (pend > 1.9 * avg)).astype(np.uint8)
    p = dict(nthreads=nth, occ=occ, nproc=nproc, wnbytes=wnbytes, idle=idle, sat=sat, total_occ=total_occ,
             total_nthreads=tn, bandwidth=bw, victim=victim, duration=duration, fast=np.zeros(T, np.uint8),
             dep_ptr=dep_ptr, dep_idx=dep_idx, data_nbytes=nbytes, data_get_nbytes=nbytes, data_holder=holder,
             **({"holder_ptr": hptr, "holder_idx": hidx} if replicas > 1 else {}))
    if restrict > 0:  # worker restrictions on a fraction of the tasks (valid sets of 1-16, some empty / loose)
        rr = np.random.default_rng(seed + 7)
        flags = np.zeros(T, np.uint8)
        rows = [[] for _ in range(T)]
        for t in np.flatnonzero(rr.random(T) < restrict):
            flags[t] = 1 | (2 if rr.random() < 0.5 else 0)
            if rr.random() >= 0.1:
                rows[t] = sorted(set(rr.integers(0, W, int(rr.integers(1, 17))).tolist()))
        rp, ri = _csr_from_rows(rows)
        p.update(restr_ptr=rp, restr_idx=ri, restr_flags=flags)
    return p
