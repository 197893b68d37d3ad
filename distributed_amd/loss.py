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
dependencies (``loss_orders``).

Pure Python over duck-typed scheduler objects: the extension calls it on the live
scheduler, ``tests/golden/gen_service.py`` on the reference, so the fixtures' order rows are
the extension's.
"""
from __future__ import annotations

LO_DEPS, LO_WAITERS = 0, 1  # dgp_events.h LossOrder kinds


def lost_results(ws, held) -> list:
    """The replicas of ``held`` (ws.has_what order) that no other worker holds."""
    return [ts for ts in held if ts.who_has == {ws}]


def cascade(ws, proc, held):
    """The tasks whose ``released -> waiting`` the loss may run -- the processing tasks, the
    lost results that are needed, their processing waiters, and every released or lost
    dependency those recompute, transitively -- in discovery order; None when one of them is
    a case the engine does not restate (an erred or forgotten dependency, a chain task without
    run_spec or with lost dependencies, an actor)."""
    lost = lost_results(ws, held)
    lostset = set(lost)
    stack = list(proc) + [ts for ts in lost if ts.who_wants or ts.waiters]
    stack += [y for ts in lost for y in (ts.waiters or ()) if y.state == "processing"]
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


def supported(s, ws, proc, held, safe) -> list | None:
    """The cascade (see ``cascade``) when dgp_lose_worker_ordered restates the loss, else None:
    no processing task that errs (KilledWorker, :5239-5265) or that nobody needs, no lost
    result without run_spec or with a queued / no-worker waiter."""
    for ts in proc:
        if (not safe and ts.suspicious + 1 > s.allowed_failures) or not (ts.waiters or ts.who_wants):
            return None
        if ts.actor or ts.has_lost_dependencies:
            return None
    for ts in lost_results(ws, held):
        if not ts.run_spec or ts.actor or ts.has_lost_dependencies:
            return None
        for d in ts.waiters or ():
            if d.state in ("queued", "no-worker"):
                return None
            if d.state == "processing" and not (d.waiters or d.who_wants):
                return None
    return cascade(ws, proc, held)


def loss_orders(tasks, index_of) -> list:
    """(task, LO_DEPS, dependencies) rows in the engine's numbering for every task of the
    cascade with two or more dependencies, in the order this process iterates the sets."""
    rows = []
    for t in tasks:
        deps = t.dependencies
        if len(deps) >= 2:
            rows.append((index_of(t), LO_DEPS, [index_of(d) for d in deps]))
    return rows
