"""Which worker losses the engine decides itself, and the scheduler's iteration orders it needs.

``Scheduler.remove_worker`` (distributed/scheduler.py:5180-5303) recommends every processing
task of the worker and every result it held alone to "released"; the transitions that follow
(``processing -> released -> waiting``, ``memory -> released -> waiting``, ``waiting ->
processing``) are restated on the device by ``dgp_lose_worker_ordered`` (dgp_events.h). A
task re-waited there recomputes each released dependency in turn
(``_transition_released_waiting`` :2101-2106), back to results still in memory: a recompute
chain. Those recommendations enter the dict in ``ts.dependencies`` order -- a set, hashed by
key -- and the dict is popped LIFO, so the order in which the chain's tasks are placed is the
set's. The host passes that order for every task of the cascade with two or more
dependencies (``loss_orders``). A processing task out of retries errs at once
(KilledWorker, :5239-5265), and its waiting dependents with it (``erred_closure``).

Pure Python over duck-typed scheduler objects: the extension calls it on the live
scheduler, ``tests/golden/gen_service.py`` on the reference, so the fixtures' order rows are
the extension's.
"""
from __future__ import annotations

LO_DEPS, LO_WAITERS, LO_DEPENDENTS = 0, 1, 2  # dgp_events.h LossOrder kinds


def killed_flags(s, proc, safe) -> list:
    """Per processing task: it runs out of retries with this loss (KilledWorker,
    scheduler.py:5239-5265: suspicious + 1 > allowed_failures when not safe)."""
    return [bool(not safe and ts.suspicious + 1 > s.allowed_failures) for ts in proc]


def erred_closure(killed, lost=frozenset()) -> list | None:
    """The tasks the KilledWorker transitions err (each killed task, then every dependent
    without a replica, transitively: :2711-2713, :2518-2521), killed ones first; None when the
    engine does not restate that cascade -- a member besides the killed ones that is not
    waiting, or a dependency it would release that is not in memory (its waiters all erred,
    not wanted) or is a lost result (``lost``: recomputed first, then released by the erred
    waiter -- a cascade the engine refuses)."""
    out, seen, stack = list(killed), set(killed), list(killed)
    while stack:
        x = stack.pop()
        for y in x.dependents:
            if y not in seen and not y.who_has:
                seen.add(y)
                out.append(y)
                stack.append(y)
    for x in out[len(killed):]:
        if x.state != "waiting":
            return None
    for x in out:
        for d in x.dependencies:
            if d in seen:
                continue
            if not (d.waiters or set()) - seen and not d.who_wants and (d.state != "memory" or d in lost):
                return None
    return out


def lost_results(ws, held) -> list:
    """The replicas of ``held`` (ws.has_what order) that no other worker holds."""
    return [ts for ts in held if ts.who_has == {ws}]


def cascade(ws, proc, held, killed=()):
    """The tasks whose ``released -> waiting`` the loss may run -- the processing tasks, the
    lost results that are needed, their processing / no-worker waiters, and every released or lost
    dependency those recompute, transitively -- in discovery order; None when one of them is
    a case the engine does not restate (an erred or forgotten dependency, a chain task without
    run_spec or with lost dependencies, an actor)."""
    lost = lost_results(ws, held)
    lostset = set(lost)
    stack = [ts for ts in proc if ts not in killed] + [ts for ts in lost if ts.who_wants or ts.waiters]
    stack += [y for ts in lost for y in (ts.waiters or ()) if y.state in ("processing", "no-worker") and y not in killed]
    out, seen = [], set()
    while stack:
        t = stack.pop()
        if t in seen:
            continue
        seen.add(t)
        out.append(t)
        for d in t.dependencies:
            if d.state in ("erred", "forgotten"):
                return None
            if d in lostset or d.state == "released":
                if not d.run_spec or d.actor or d.has_lost_dependencies:
                    return None
                stack.append(d)
    return out


def supported(s, ws, proc, held, safe) -> tuple | None:
    """(the re-wait cascade, the erred closure) when dgp_lose_worker_ordered restates the
    loss (see ``cascade`` / ``erred_closure``), else None: no processing task that nobody
    needs, no KilledWorker cascade outside ``erred_closure``, no lost result without run_spec,
    with a queued waiter, or with a processing / no-worker waiter nobody needs (its release
    would release its own dependencies)."""
    kf = killed_flags(s, proc, safe)
    killed = [ts for ts, k in zip(proc, kf) if k]
    for ts, k in zip(proc, kf):
        if ts.actor or ts.has_lost_dependencies:
            return None
        if not k and not (ts.waiters or ts.who_wants):
            return None
    ks = set(killed)
    for ts in lost_results(ws, held):
        if not ts.run_spec or ts.actor or ts.has_lost_dependencies:
            return None
        for d in ts.waiters or ():
            if d in ks:
                continue
            if d.state == "queued":  # leaves ts.waiters at the recompute yet stays queued
                return None
            if d.state in ("processing", "no-worker") and not (d.waiters or d.who_wants):
                return None
    erred = erred_closure(killed, set(lost_results(ws, held))) if killed else []
    if erred is None:
        return None
    chain = cascade(ws, proc, held, ks)
    if chain is None or set(chain) & set(erred):
        return None
    return chain, erred


def loss_orders(tasks, index_of, erred=(), n_killed=0) -> list:
    """The (task, kind, tasks) rows in the engine's numbering, in the order this process
    iterates the sets: LO_DEPS for every task of the re-wait cascade and of the erred closure
    with two or more dependencies; for the erred closure also LO_WAITERS of each killed task
    (its first ``n_killed``) and LO_DEPENDENTS of the others, with two or more members."""
    rows = []
    for t in list(tasks) + list(erred):
        deps = t.dependencies
        if len(deps) >= 2:
            rows.append((index_of(t), LO_DEPS, [index_of(d) for d in deps]))
    for i, t in enumerate(erred):
        kin = (LO_WAITERS, t.waiters or ()) if i < n_killed else (LO_DEPENDENTS, t.dependents)
        if len(kin[1]) >= 2:
            rows.append((index_of(t), kin[0], [index_of(y) for y in kin[1]]))
    return rows


def graph_cascade(new) -> list | None:
    """A later graph's update_graph stimulus (scheduler.py:4598-4611): the earlier tasks its
    runnable ``new`` tasks recompute -- released dependencies, transitively back to results in
    memory (:2105-2106) -- in discovery order; None when the engine does not restate the
    stimulus (an erred, forgotten or blamed dependency: the new task errs, :4613-4618; a task
    to recompute without run_spec, with lost dependencies or an actor)."""
    newset = set(new)
    out, seen, stack = [], set(), list(new)
    while stack:
        t = stack.pop()
        for d in t.dependencies:
            if d in newset or d in seen:
                continue
            if d.state in ("erred", "forgotten") or d.exception_blame:
                return None
            if d.state == "released":
                if not d.run_spec or d.actor or d.has_lost_dependencies:
                    return None
                seen.add(d)
                out.append(d)
                stack.append(d)
    return out


def graph_orders(new, chain, index_of) -> list:
    """(task, LO_DEPS, dependencies) rows for the tasks of a later graph's stimulus whose
    recommendations follow a set: a new or recomputed task with two or more dependencies that
    are recomputed (the others are either in the dict already -- the new ones, whose place
    stays -- or only gain it as a waiter)."""
    cs = set(chain)
    return [(index_of(t), LO_DEPS, [index_of(d) for d in t.dependencies])
            for t in list(new) + list(chain) if sum(d in cs for d in t.dependencies) >= 2]


class _NotModelled(Exception):
    pass


def release_plan(s, client, keys) -> list | None:
    """client-releases-keys (scheduler.py:5417-5430): every task its transitions reach, each
    with its forget flag, in the order the scheduler runs them (dgp_release_tasks applies them
    in that order). _client_releases_keys (:3400-3419) recommends the keys no other client
    wants -- forgotten without dependents, else released when nothing waits on them -- and
    SchedulerState._transitions pops that dict LIFO, merging what each transition recommends
    (dict.update: a key already present keeps its place). Restated here on a shadow of the
    states, waiters, dependents and who_wants it changes:

      memory -> released       :2444-2505    processing -> released  :2606-2628 (+ :3337-3357)
      waiting -> released      :2579-2604    queued / no-worker -> released  :2784-2795, :2747-2759
      released / memory -> forgotten  :2853-2881, :2821-2851 (_propagate_forgotten :3359-3398)
      anything else -> released first, then on (:1961-1984)

    None when the release reaches a case the engine does not restate: a task re-waited (a
    released task something still needs), an erred or actor task, a forgotten task whose
    dependents would be flagged with lost dependencies, a cancelled task that is not in one of
    its dependencies' waiters: the scheduler's stimulus, then a resync."""
    cs = s.clients.get(client)
    if cs is None:
        return []
    recs, wants = {}, {}
    for key in keys:
        ts = s.tasks.get(key)
        if ts is None or ts in wants or ts not in (cs.wants_what or ()):
            continue
        left = set(ts.who_wants or ()) - {cs}
        wants[ts] = left
        if left:
            continue  # still wanted by another client: who_wants changes, nothing transitions
        if not ts.dependents:
            recs[ts] = "forgotten"
        elif ts.state != "erred" and not ts.waiters:
            recs[ts] = "released"
    state, wset, dset = {}, {}, {}

    def st(ts):
        return state.get(ts, ts.state)

    def waiters(ts):
        if ts not in wset:
            wset[ts] = set(ts.waiters or ())
        return wset[ts]

    def dependents(ts):
        if ts not in dset:
            dset[ts] = set(ts.dependents)
        return dset[ts]

    def who(ts):
        return wants[ts] if ts in wants else (ts.who_wants or set())

    ops, forget = {}, set()

    def leave_waiters(ts, r):  # a cancelled task leaves its dependencies' waiters
        for dts in ts.dependencies:
            if st(dts) == "released":
                continue
            w = waiters(dts)
            if ts not in w:
                raise _NotModelled  # the engine's count would drop a task the set never held
            w.discard(ts)
            if not w and not who(dts):
                r[dts] = "released"

    def propagate_released(ts, r):  # :3337-3357
        state[ts] = "released"
        if ts.has_lost_dependencies:
            r[ts] = "forgotten"
        elif waiters(ts) or who(ts):
            raise _NotModelled  # re-waited
        leave_waiters(ts, r)
        wset[ts] = set()

    def to_released(ts, start):
        r = {}
        if ts.actor:
            raise _NotModelled
        ops.setdefault(ts, None)
        if start == "memory":
            state[ts] = "released"
            if not ts.run_spec or ts.has_lost_dependencies:
                r[ts] = "forgotten"
            elif who(ts) or waiters(ts):
                raise _NotModelled  # re-waited (and its waiters' recommendations)
        elif start in ("processing", "queued", "no-worker"):
            propagate_released(ts, r)
        elif start == "waiting":
            for dts in ts.dependencies:
                w = waiters(dts)
                if ts in w:
                    w.discard(ts)
                    if not w and not who(dts):
                        r[dts] = "released"
                elif st(dts) != "released":
                    raise _NotModelled
            state[ts] = "released"
            if ts.has_lost_dependencies:
                r[ts] = "forgotten"
            elif not ts.exception_blame and (who(ts) or waiters(ts)):
                raise _NotModelled
            wset[ts] = set()
        else:
            raise _NotModelled
        return r

    def to_forgotten(ts):  # :2853-2881 / :2821-2851 -> _propagate_forgotten (a result's replicas go)
        if ts.actor or dependents(ts):
            raise _NotModelled  # its dependents would be flagged with lost dependencies
        ops.setdefault(ts, None)
        forget.add(ts)
        r = {}
        for dts in ts.dependencies:
            dependents(dts).discard(ts)
            waiters(dts).discard(ts)
            if not dependents(dts) and not who(dts):
                r[dts] = "forgotten"
        state[ts] = "forgotten"
        return r

    def transition(ts, finish):  # SchedulerState._transition :1910-1990
        start = st(ts)
        if start == "forgotten" or start == finish:
            return {}
        if finish == "released":
            return to_released(ts, start)
        if finish == "forgotten":
            if start in ("released", "memory"):
                return to_forgotten(ts)
            a = to_released(ts, start)
            v = a.get(ts, finish)
            if v != "forgotten":
                raise _NotModelled
            b = to_forgotten(ts)
            a.update(b)
            return a
        raise _NotModelled

    try:
        while recs:
            ts, finish = recs.popitem()
            recs.update(transition(ts, finish))
    except _NotModelled:
        return None
    return [(ts, ts in forget) for ts in ops]
