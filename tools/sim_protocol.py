"""Critical-path model of the C2 replay under two executor protocols (diagnostics, CPU).

Stimulus r completes placement r (the replay order). It touches its completing worker w,
the holders of the dependencies it releases (only ws.nbytes changes) and, for each task it
makes ready (its frontier, ascending priority), the holders of that task's dependencies
(decide_worker's candidates; the chosen one is written). Workers are ordered resources:
a stimulus may use worker c once every earlier stimulus that touches c has released it.

  A  "claim when all touched workers are free" (the current k_stream protocol): release-only
     holders are released after the completion, non-chosen candidates after the last
     decision, chosen candidates after the frontier, w at the end.
  B  "claim when w is free, wait in place": the completion runs on w alone; each decision
     waits for its own candidates (spinning on their release), a candidate is released
     after the last decision that reads it (the chosen one after its commit).

Unlimited executors: the replay time is the latest finish (a lower bound). Costs in cycles
(--costs), defaults from the DGP_TRACE=2 phase trace.
    python tools/sim_protocol.py [n_tasks] [--costs claim,compl,rel,dec,commit,end,spin]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs  # noqa: E402
from oracle import oracle  # noqa: E402


def structure(n, w):
    g = graphs.random_dag(n, w, seed=0)
    ref = oracle.replay(g, {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5,
                            "saturation": 1.1}, snapshots=False)
    pt, pw = ref["pl_task"], ref["pl_worker"]
    N = g["n_tasks"]
    run = np.full(N, -1, np.int64)
    run[pt] = np.arange(len(pt))
    holder = np.full(N, -1, np.int64)
    holder[pt] = pw
    dp, di = g["dep_ptr"], g["dep_idx"]
    k = np.diff(dp)
    xs = np.repeat(np.arange(N), k)
    fr = np.full(N, -1, np.int64)
    np.maximum.at(fr, xs, run[di])
    rel = np.full(N, -1, np.int64)
    np.maximum.at(rel, di, run[xs])
    hasdep = np.zeros(N, bool)
    hasdep[di] = True
    relmask = hasdep & (g["wanted"] == 0) & (rel >= 0)
    return g, pt, pw, run, holder, fr, rel, relmask


def simulate(S, costs, mode, n_exe=0):
    g, pt, pw, run, holder, fr, rel, relmask = S
    claim, compl, trel, dec, commit, end, spin = costs
    N = g["n_tasks"]
    dp, di = g["dep_ptr"], g["dep_idx"]
    # per stimulus: frontier tasks (ascending priority = ascending index here), releases
    order = np.argsort(fr, kind="stable")
    frs = fr[order]
    fptr = np.searchsorted(frs, np.arange(len(pt) + 1))
    rels = np.nonzero(relmask)[0]
    rel_r = rel[rels]
    ro = np.argsort(rel_r, kind="stable")
    rels, rel_r = rels[ro], rel_r[ro]
    rptr = np.searchsorted(rel_r, np.arange(len(pt) + 1))
    free = np.zeros(int(pw.max()) + 1)
    finish = 0.0
    import heapq
    exe = [0.0] * n_exe  # executor free times (n_exe = 0: unlimited)
    last_claim = 0.0
    for r in range(len(pt)):
        w = int(pw[r])
        F = order[fptr[r]:fptr[r + 1]]
        F = F[F != pt[r]]
        R = [int(holder[d]) for d in rels[rptr[r]:rptr[r + 1]]]
        cands = [[int(holder[d]) for d in di[dp[x]:dp[x + 1]]] for x in F]
        chosen = [int(holder[x]) for x in F]
        e0 = heapq.heappop(exe) if n_exe else 0.0
        if mode == "A":
            touched = {w, *R, *[c for cs in cands for c in cs]}
            t = max(max(free[c] for c in touched), e0) + claim
            t += compl
            t += trel
            for c in R:
                if c != w and all(c not in cs for cs in cands):
                    free[c] = t
            t_dec = t + dec * len(F)
            t_end_f = t_dec + commit * len(F)
            for c in touched:
                if c == w or c in R and all(c not in cs for cs in cands):
                    continue
                free[c] = t_end_f if c in chosen else t_dec
            t = t_end_f + end
            free[w] = t
        else:
            t0 = max(e0, last_claim)  # in-order claims
            last_claim = t0
            t = max(free[w] + spin, t0 + claim) + compl + trel
            held = {w}
            for c in R:
                if c == w:
                    continue
                t2 = max(t, free[c] + spin)
                free[c] = t2 + 50  # an nbytes add, released at once
            last_use = {}
            for j, cs in enumerate(cands):
                for c in cs:
                    last_use[c] = j
            for j, cs in enumerate(cands):
                need = [c for c in cs if c not in held]
                if need:
                    t = max(t, max(free[c] + spin for c in need))
                    held.update(need)
                t += dec
                b = chosen[j]
                for c in cs:
                    if c != b and c != w and last_use[c] == j and c not in chosen[j + 1:]:
                        free[c] = t
                t += commit
                if b != w and last_use.get(b, -1) == j:
                    free[b] = t
            t += end
            free[w] = t
        finish = max(finish, t)
        if n_exe:
            heapq.heappush(exe, t)
    return finish


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 1_000_000
    costs = [3000, 5000, 500, 1500, 2500, 2000, 300]
    if "--costs" in sys.argv:
        costs = [float(x) for x in sys.argv[sys.argv.index("--costs") + 1].split(",")]
    S = structure(n, 1024)
    for n_exe in (0, 8, 11, 16, 24):
        for mode in ("A", "B"):
            f = simulate(S, costs, mode, n_exe)
            print(f"executors {n_exe or 'inf':>3} mode {mode}: {f / 2.4e9 * 1e3:7.1f} ms at 2.4 GHz; "
                  f"{n / (f / 2.4e9) / 1e6:.2f} M/s")


if __name__ == "__main__":
    main()
