"""The engine's task prefix table over a scheduler session.

The stream engine carries at most ``PX`` task prefixes (``dgp_stream.h``), while a long-lived
scheduler meets one ``TaskPrefix`` per ``key_split`` name for its whole session
(``distributed/scheduler.py:923-1031``, ``SchedulerState.task_prefixes``). Only the live
prefixes matter to placement: those of the tasks that are waiting, queued, processing or
no-worker and those counted in a worker's or the global ``task_prefix_count``
(``_calc_occupancy`` :1884-1903 sums exactly these). A task of any other prefix is released,
in memory, erred or forgotten: nothing reads its prefix until it is recomputed, and every
recompute the engine does not run itself (a later graph that needs a released task) is the
scheduler's stimulus followed by a resync, which makes the table current again first
(``GPUPlacementExtension._prefixes_current``); the recomputes the engine runs itself
(``dgp_lose_worker_ordered``, recompute chains included) are only offered when every task of
the cascade has its prefix's slot.

So when a later graph would pass ``PX`` prefixes, the table is compacted: the live prefixes
keep their relative order, the new graph's follow, and ``dgp_remap_prefixes`` gives every
engine task its slot in the new table (a dead prefix's tasks get slot 0, never read), after
which ``dgp_sync_workers`` / ``dgp_sync_globals`` bring the dicts, durations and queue in the
new numbering. Pure Python over duck-typed scheduler objects: the extension calls it on the
live scheduler, ``tests/golden/gen_service.py`` on the reference replay state, so the
fixtures' remaps are the extension's.
"""
from __future__ import annotations

import numpy as np

PX = 32  # dgp_stream.h PX
LIVE_STATES = ("waiting", "queued", "processing", "no-worker")


def live_prefixes(s) -> set:
    """The prefix names placement may still read (see the module docstring)."""
    live = set(getattr(s, "_task_prefix_count_global", {}) or {})
    for ws in s.workers.values():
        live.update(ws.task_prefix_count)
    for nm, tp in s.task_prefixes.items():
        st = tp.states
        if any(st.get(k, 0) for k in LIVE_STATES):
            live.add(nm)
    return live


def compacted(slot_of: dict, live: set, extra) -> dict | None:
    """The new name -> slot table: the live names that had a slot in their old order, the
    other live names by name, then ``extra`` (a new graph's prefix names, in its order) not
    yet placed; None when that is more than PX."""
    kept = sorted((nm for nm in live if nm in slot_of), key=slot_of.__getitem__)
    kept += sorted(nm for nm in live if nm not in slot_of)
    seen = set(kept)
    for nm in extra:
        if nm not in seen:
            kept.append(nm)
            seen.add(nm)
    if len(kept) > PX:
        return None
    return {nm: i for i, nm in enumerate(kept)}


def task_slots(task_names: np.ndarray, names: list, slot_of: dict) -> tuple[np.ndarray, np.ndarray]:
    """(every engine task's slot, the tasks left without one): ``task_names`` holds each
    task's prefix as an index into ``names``."""
    lut = np.array([slot_of.get(nm, -1) for nm in names] or [-1], np.int32)
    s = lut[np.asarray(task_names, np.int64)] if len(task_names) else np.zeros(0, np.int32)
    stale = np.flatnonzero(s < 0)
    s = np.where(s < 0, 0, s).astype(np.int32)
    return s, stale
