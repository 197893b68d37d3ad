"""Host-side model of the compute-task message fields of a batch of placements (test
infrastructure: the checker of tests/ext_driver.py and tests/test_messages.py; the
product builds them from dgp_task_messages, distributed_amd/ext.py _engine_task_msg).

The reference builds one dict per placement in ``SchedulerState._task_to_msg``
(scheduler.py:3421-3450): ``who_has`` / ``nbytes`` of every dependency, the task's
``priority`` and ``run_id``, its ``duration``. After the engine placed a batch, the
same fields for the whole batch come from arrays: the placement log (which worker
each dependency ran on: its only replica in this protocol, ``add_replica`` :3148),
the graph CSR and the result sizes the task-finished messages reported
(``TaskState.nbytes``, raw, as ``_task_to_msg`` sends it). ``compute_task_batch``
gathers them with numpy in one pass (columnar, CSR by placement);
``render_messages`` turns rows into the reference's message dicts.

``duration`` is the caller's (TaskPrefix.duration_average at render time, or the
unknown-task default): the reference notes the worker does not use it (:3423-3424).
"""
from __future__ import annotations

import numpy as np


def compute_task_batch(g: dict, pl_task: np.ndarray, pl_worker: np.ndarray, offset: int, count: int,
                       nbytes: np.ndarray) -> dict:
    """Columnar compute-task fields of placements [offset, offset + count) of a placement
    log (``pl_task`` / ``pl_worker``: the whole log so far, in placement order).

    Returns ``task`` / ``worker`` [count], ``run_id`` [count] (the placement index), and
    the dependencies as CSR ``dep_ptr`` [count + 1] / ``dep_task`` / ``dep_holder`` /
    ``dep_nbytes`` (holder = the worker the dependency was placed on and completed on;
    nbytes = its reported size, -1 if it reported none)."""
    pl_task = np.asarray(pl_task, np.int64)
    pl_worker = np.asarray(pl_worker, np.int32)
    n = int(g["n_tasks"])
    if not 0 <= offset <= offset + count <= len(pl_task):
        raise ValueError(f"compute_task_batch: [{offset}, {offset + count}) outside the log ({len(pl_task)})")
    holder = np.full(n, -1, np.int32)
    holder[pl_task[: offset + count]] = pl_worker[: offset + count]
    tasks = pl_task[offset: offset + count]
    dp = np.asarray(g["dep_ptr"], np.int64)
    di = np.asarray(g["dep_idx"], np.int64)
    k = dp[tasks + 1] - dp[tasks]
    ptr = np.zeros(count + 1, np.int64)
    np.cumsum(k, out=ptr[1:])
    # every dependency edge of the batch, in CSR order: starts repeated, plus the offset in the row
    starts = np.repeat(dp[tasks], k)
    within = np.arange(int(ptr[-1]), dtype=np.int64) - np.repeat(ptr[:-1], k)
    dep = di[starts + within]
    if len(dep) and (holder[dep] < 0).any():
        raise ValueError("compute_task_batch: a dependency of the batch was never placed")
    return dict(task=tasks.astype(np.int32), worker=pl_worker[offset: offset + count].copy(),
                run_id=np.arange(offset, offset + count, dtype=np.int64), dep_ptr=ptr,
                dep_task=dep.astype(np.int32), dep_holder=holder[dep], dep_nbytes=np.asarray(nbytes, np.int64)[dep])


def render_messages(batch: dict, keys, addresses, priority, duration) -> list:
    """The batch as ``_task_to_msg``-shaped dicts (op, key, run_id, priority, duration,
    who_has, nbytes); ``keys`` / ``addresses`` map task / worker indices to names,
    ``priority(i)`` / ``duration(i)`` give a task's priority tuple and duration."""
    out = []
    ptr = batch["dep_ptr"]
    for j, t in enumerate(batch["task"].tolist()):
        a, b = int(ptr[j]), int(ptr[j + 1])
        deps = batch["dep_task"][a:b].tolist()
        hold = batch["dep_holder"][a:b].tolist()
        nb = batch["dep_nbytes"][a:b].tolist()
        out.append({
            "op": "compute-task", "key": keys[t], "run_id": int(batch["run_id"][j]), "priority": priority(t),
            "duration": duration(t),
            "who_has": {keys[d]: [addresses[h]] for d, h in zip(deps, hold)},
            "nbytes": {keys[d]: x for d, x in zip(deps, nb)},
        })
    return out
