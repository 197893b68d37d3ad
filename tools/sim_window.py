"""Offline model of the stream engine's schedule (diagnostic, CPU only).

From the oracle's placement log of a replay, build every stimulus' touch set (completing
worker, release holders, frontier-candidate holders), then simulate in-order registration
into a window of WIN slots, start = all earlier stimuli sharing a worker finished,
in-order retirement, E executors of latency L (µs), registrar cost R (µs/stimulus).
Prints the modelled placements/s, to tell window-bound from latency-bound regimes.

    python tools/sim_window.py [n_tasks] [n_workers]
"""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs  # noqa: E402
from oracle import oracle  # noqa: E402

CFG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}


def touch_sets(g, pl_task, pl_worker):
    n = g["n_tasks"]
    run_id = np.empty(n, np.int64)
    run_id[pl_task] = np.arange(len(pl_task))
    holder = np.empty(n, np.int64)
    holder[pl_task] = pl_worker
    dp, di = g["dep_ptr"].astype(np.int64), g["dep_idx"].astype(np.int64)
    k = np.diff(dp)
    src = np.repeat(np.arange(n), k)
    # frontier mark: the stimulus completing x's last dependency
    fr = np.full(n, -1, np.int64)
    np.maximum.at(fr, src, run_id[di])
    # release mark: the stimulus completing d's last dependent (not wanted)
    rel = np.full(n, -1, np.int64)
    np.maximum.at(rel, di, run_id[src])
    wanted = g["wanted"].astype(bool)
    nodep = np.bincount(di, minlength=n) == 0
    rel[wanted] = -1
    rel[nodep] = -1
    pairs_r = [np.arange(len(pl_task))]
    pairs_w = [pl_worker.astype(np.int64)]
    m = rel >= 0
    pairs_r.append(rel[m])
    pairs_w.append(holder[m])
    fx = k > 0
    e_fr = np.repeat(fr, k)  # per dependency edge: the frontier stimulus of its task
    pairs_r.append(e_fr[np.repeat(fx, k)])
    pairs_w.append(holder[di][np.repeat(fx, k)])
    R = np.concatenate(pairs_r)
    Wk = np.concatenate(pairs_w)
    key = np.unique(R * (1 << 20) + Wk)
    R, Wk = key >> 20, key & ((1 << 20) - 1)
    ptr = np.searchsorted(R, np.arange(len(pl_task) + 1))
    return ptr, Wk


def touch_roles(g, pl_task, pl_worker, ptr, wk):
    """frac[k]: when (fraction of the execution) stimulus ptr-row releases worker wk[k]:
    1.0 for the completing worker and chosen workers, 0.5 for workers only read as
    candidates or only adjusted as release holders."""
    n = g["n_tasks"]
    run_id = np.empty(n, np.int64)
    run_id[pl_task] = np.arange(len(pl_task))
    dp, di = g["dep_ptr"].astype(np.int64), g["dep_idx"].astype(np.int64)
    k = np.diff(dp)
    src = np.repeat(np.arange(n), k)
    fr = np.full(n, -1, np.int64)
    np.maximum.at(fr, src, run_id[di])
    chosen = pl_worker[run_id]  # worker each task was placed on
    R = np.repeat(np.arange(len(ptr) - 1), np.diff(ptr))
    key = set()
    m = fr >= 0
    for r_, c_ in zip(fr[m], chosen[m]):
        key.add((int(r_), int(c_)))
    frac = np.full(len(wk), 0.5)
    for i in range(len(wk)):
        r_ = int(R[i]); c_ = int(wk[i])
        if c_ == pl_worker[r_] or (r_, c_) in key:
            frac[i] = 1.0
    return frac


def simulate_early(ptr, wk, frac, n_stim, E, L, first):
    last = {}
    execs = [0.0] * E
    heapq.heapify(execs)
    tmax = 0.0
    for r in range(first, n_stim):
        st = 0.0
        a, b = ptr[r], ptr[r + 1]
        for i in range(a, b):
            v = last.get(wk[i])
            if v is not None and v > st:
                st = v
        ex = heapq.heappop(execs)
        st = max(st, ex)
        f = st + L
        heapq.heappush(execs, f)
        for i in range(a, b):
            last[wk[i]] = st + L * frac[i]
        tmax = max(tmax, f)
    return tmax


def simulate(ptr, wk, n_stim, WIN, E, L, Rc, first):
    last = {}
    fin = np.zeros(n_stim)
    seq = np.zeros(n_stim)  # retirement (in order)
    reg_t = 0.0
    execs = [0.0] * E
    heapq.heapify(execs)
    for r in range(first, n_stim):
        reg_t = reg_t + Rc
        if r - WIN >= first:
            reg_t = max(reg_t, seq[r - WIN])
        st = reg_t
        ws = wk[ptr[r]:ptr[r + 1]]
        for c in ws:
            v = last.get(c)
            if v is not None and v > st:
                st = v
        ex = heapq.heappop(execs)
        st = max(st, ex)
        f = st + L
        heapq.heappush(execs, f)
        fin[r] = f
        for c in ws:
            last[c] = f
        seq[r] = max(seq[r - 1] if r > first else 0.0, f)
    return seq[n_stim - 1]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    g = graphs.random_dag(n, W, seed=0)
    ref = oracle.replay(g, CFG, snapshots=False)
    pl_task, pl_worker = ref["pl_task"].astype(np.int64), ref["pl_worker"].astype(np.int64)
    ptr, wk = touch_sets(g, pl_task, pl_worker)
    sz = np.diff(ptr)
    print(f"{n} tasks x {W} workers: touch set mean {sz.mean():.2f} max {sz.max()}")
    first = 2 * W  # update_graph wave: not part of the stream kernel
    n_stim = len(pl_task)
    frac = touch_roles(g, pl_task, pl_worker, ptr, wk)
    print(f"early-releasable touches: {(frac < 1).mean():.2f}")
    for L in (4.0, 2.0):
        for E in (11, 32):
            t = simulate_early(ptr, wk, frac, n_stim, E, L, first)
            t0 = simulate_early(ptr, wk, np.ones_like(frac), n_stim, E, L, first)
            print(f"E {E} L {L}us: release at end {(n_stim - first) / t0:.3f} M/s, early release {(n_stim - first) / t:.3f} M/s")
    for WIN in (32,):
        for L in (8.0, 4.0, 2.0, 1.0):
            for Rc in (0.0, 0.25):
                t = simulate(ptr, wk, n_stim, WIN, 11, L, Rc, first)
                print(f"WIN {WIN:4d} L {L:4.1f}us R {Rc:4.2f}us -> {(n_stim - first) / t:8.3f} M/s")


def simulate_ooo(ptr, wk, n_stim, WIN, E, L, Rc, first, ooo=True, frac=None):
    """As simulate(), but a slot is freed when its stimulus finishes (out of order) when
    ooo, else at in-order retirement. frac: early release fractions (None: at the end)."""
    last = {}
    reg_t = 0.0
    execs = [0.0] * E
    heapq.heapify(execs)
    fin_heap = []  # finish times of registered, unfreed stimuli
    seq_prev = 0.0
    retire = []
    for r in range(first, n_stim):
        reg_t = reg_t + Rc
        if ooo:
            while len(fin_heap) >= WIN:
                reg_t = max(reg_t, heapq.heappop(fin_heap))
        elif r - WIN >= first:
            reg_t = max(reg_t, retire[r - WIN - first])
        st = reg_t
        a, b = ptr[r], ptr[r + 1]
        for i in range(a, b):
            v = last.get(wk[i])
            if v is not None and v > st:
                st = v
        ex = heapq.heappop(execs)
        st = max(st, ex)
        f = st + L
        heapq.heappush(execs, f)
        for i in range(a, b):
            last[wk[i]] = st + L * (frac[i] if frac is not None else 1.0)
        if ooo:
            heapq.heappush(fin_heap, f)
        seq_prev = max(seq_prev, f)
        retire.append(seq_prev)
    return seq_prev


def main_ooo():
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
    W = 1024
    g = graphs.random_dag(n, W, seed=0)
    ref = oracle.replay(g, CFG, snapshots=False)
    pl_task, pl_worker = ref["pl_task"].astype(np.int64), ref["pl_worker"].astype(np.int64)
    ptr, wk = touch_sets(g, pl_task, pl_worker)
    frac = touch_roles(g, pl_task, pl_worker, ptr, wk)
    first = 2 * W
    n_stim = len(pl_task)
    for L in (5.3, 4.0, 2.5):
        for E in (7, 11):
            for WIN in (32, 64):
                for Rc in (0.7, 0.35):
                    t_in = simulate_ooo(ptr, wk, n_stim, WIN, E, L, Rc, first, ooo=False, frac=frac)
                    t_oo = simulate_ooo(ptr, wk, n_stim, WIN, E, L, Rc, first, ooo=True, frac=frac)
                    print(f"L {L} E {E} WIN {WIN} R {Rc}: in-order {(n_stim - first) / t_in:.3f} M/s, out-of-order slots {(n_stim - first) / t_oo:.3f} M/s", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ooo":
        main_ooo()
    else:
        main()
