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


def release_plan(s, client, keys) -> list | None:
    """client-releases-keys (scheduler.py:5417-5430): the tasks its transitions reach, each
    with its forget flag -- the keys no other client wants (_client_releases_keys
    :3400-3419: forgotten without dependents, else released when nothing waits on them), then
    every dependency _propagate_forgotten forgets (:3378-3385: no dependent left, not wanted)
    -- when all of them are results in memory or released (dgp_release_tasks); None when
    the release reaches anything else (a cancellation, an erred or actor task, a forgotten
    task with dependents still live): the scheduler's stimulus, then a resync."""
    cs = s.clients.get(client)
    if cs is None:
        return []
    recs, seen = [], set()
    for key in keys:
        ts = s.tasks.get(key)
        if ts is None or ts in seen or ts not in (cs.wants_what or ()):
            continue
        seen.add(ts)
        if (ts.who_wants or set()) - {cs}:
            continue  # still wanted by another client: who_wants changes, nothing transitions
        if not ts.dependents:
            recs.append((ts, True))
        elif ts.state != "erred" and not ts.waiters:
            recs.append((ts, False))
    plan, forgotten, stack = {}, set(), list(recs)
    while stack:
        ts, forget = stack.pop()
        if ts.state not in ("memory", "released") or ts.actor:
            return None
        if not forget and (not ts.run_spec or ts.has_lost_dependencies):
            forget = True  # memory -> released of pure data / lost dependencies: forgotten (:2485-2488)
        if not forget:
            plan.setdefault(ts, False)
            continue
        if ts in forgotten:
            continue
        forgotten.add(ts)
        plan[ts] = True
        if any(d not in forgotten for d in ts.dependents):
            return None  # its dependents would be forgotten or flagged with lost dependencies
        for dts in ts.dependencies:
            if not any(x not in forgotten for x in dts.dependents) and not dts.who_wants:
                stack.append((dts, True))
    return list(plan.items())
