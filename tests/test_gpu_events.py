"""Service events (needs an MI355X): the placement-input stimuli a live scheduler handles
besides task-finished, on the device, against the reference's own handlers.

The ``svcev_*`` fixtures (``tests/golden/gen_service.py events``) run the replay protocol's
task-finished messages through ``Scheduler.stimulus_task_finished`` with, interleaved and
each through the reference's handler: add-keys (``Scheduler.add_keys`` -> ``add_replica``,
distributed/scheduler.py:7359-7391, :3148), release-worker-data (:5807-5815, never the
last replica), worker pause / resume (``handle_worker_status_change`` :5850-5883),
long-running (``handle_long_running`` :5817-5848), heartbeats (the bandwidth EWMA
:4223-4226 and ``TaskPrefix.add_exec_time`` :4247-4252) and task-erred
(``handle_task_erred`` :5799-5805). Each event goes to its engine call
(``dgp_add_replicas`` / ``dgp_remove_replicas`` / ``dgp_set_worker_status`` /
``dgp_long_running`` / ``dgp_heartbeat`` / ``dgp_task_erred``) before the message it preceded
in the reference; every placement (task, worker, comm bytes, objective bits, ws.nbytes,
route), the placements each event made, the per-round snapshots and the final task states
must equal the reference's.
"""
import os

import numpy as np
import pytest

from conftest import (GOLDEN, second_graph, svc_dep_graph_files, svc_event_files, svc_p2p_files, svc_prio_graph_files,
                      svc_loss_files, svc_release_files, svc_restr_graph_files, svc_resync_files, svc_retire_files,
                      svc_retry_files)
from oracle import oracle
from test_gpu_parity import PL_KEYS, ROUND_KEYS, assert_same

pytestmark = pytest.mark.gpu

EV_FINISHED, EV_ADD_KEYS, EV_RELEASE_DATA, EV_PAUSE, EV_RESUME, EV_LONG_RUNNING, EV_HEARTBEAT, EV_ERRED = range(8)
EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS = 8, 9, 10
EV_SHUFFLE_INIT, EV_RESTRICT = 11, 12
EV_RETIRE, EV_RETIRE_REPLICA = 13, 14
EV_LOSE_WORKER = 15
EV_ERRED_RETRY, EV_REFILL = 16, 17


def sync_dump(z, j):
    """Resync rows number j of a svcrs_* fixture (gen_service.py _pack_dumps)."""
    out = {"tasks": {}, "workers": {}, "globals": {}}
    for k in z.files:
        if not k.startswith("sync_") or (k.endswith("_ptr") and k[:-4] in z.files):
            continue  # a field's per-dump offsets
        part, field = k[5:].split("_", 1)
        p = z[k + "_ptr"]
        v = z[k][p[j]:p[j + 1]]
        out[part][field] = v[0] if part == "globals" and field in ("n_tasks", "network_occ_global", "bandwidth") else v
    return out


def loss_order_rows(z, i):
    """The set-order rows of loss event i (svcwl_chain_*: gen_service.py records what
    distributed_amd.loss.loss_orders gave in the generating process), as (task, kind, tasks)."""
    if "lo_evptr" not in z.files:
        return ()
    ep, rp, idx = z["lo_evptr"], z["lo_rowptr"], z["lo_idx"]
    return [(int(z["lo_task"][r]), int(z["lo_kind"][r]), idx[rp[r]:rp[r + 1]].tolist()) for r in range(ep[i], ep[i + 1])]


def graph_order_rows(z):
    """The set-order rows of a svcgrec_* later graph's recompute (None: a plain stimulus)."""
    if "g2_lo_task" not in z.files:
        return None
    rp, idx = z["g2_lo_rowptr"], z["g2_lo_idx"]
    return [(int(t), int(k), idx[rp[r]:rp[r + 1]].tolist())
            for r, (t, k) in enumerate(zip(z["g2_lo_task"].tolist(), z["g2_lo_kind"].tolist()))]


def loss_killed(z, i, proc):
    """Per processing task of loss event i: it ran out of retries (svcwl_killed_*)."""
    if "lo_kptr" not in z.files:
        return None
    k = set(z["lo_ktask"][z["lo_kptr"][i]:z["lo_kptr"][i + 1]].tolist())
    return [int(t) in k for t in proc]


def drive_events(eng, g, z, exp=None, device_resched=False, device_release=False, release_states=None):
    """Every event of a svcev_* stream through the engine, snapshot per round; returns the
    placements each event made (update_graph's first)."""
    kind, task, worker, x = z["ev_kind"], z["ev_task"], z["ev_worker"], z["ev_x"]
    hp, ht, hd = z["hb_ptr"], z["hb_task"], z["hb_dur"]
    ptr = z["ev_round_ptr"].tolist()
    stim = [eng.num_placements()]
    n_sync = 0
    for k in range(len(ptr) - 1):
        for i in range(ptr[k], ptr[k + 1]):
            n0 = eng.num_placements()
            kd, t, w = int(kind[i]), int(task[i]), int(worker[i])
            if kd == EV_FINISHED:
                st, _ = eng.tasks_finished([t], [w], [int(z["ev_runid"][i])], [int(z["ev_nbytes"][i])],
                                           [float(z["ev_start"][i])], [float(z["ev_stop"][i])])
                assert st.tolist() == [0], (i, st)
            elif kd == EV_ADD_KEYS:
                eng.add_replicas([t], [w])
            elif kd == EV_RELEASE_DATA:
                eng.remove_replicas([t], [w])
            elif kd in (EV_PAUSE, EV_RESUME):
                eng.set_worker_status(w, 1 if kd == EV_RESUME else 0)
            elif kd == EV_LONG_RUNNING:
                eng.long_running(t, float(x[i]))
            elif kd == EV_HEARTBEAT:
                ts = ht[hp[i]:hp[i + 1]]
                eng.heartbeat(float(x[i]), g["prefix_id"][ts], hd[hp[i]:hp[i + 1]])
            elif kd == EV_ERRED:
                eng.task_erred(t)
            elif kd == EV_SHUFFLE_INIT:  # _ensure_output_tasks_are_non_rootish: the unpacks' _rootish False
                ts = ht[hp[i]:hp[i + 1]]
                eng.set_rootish(ts, np.zeros(len(ts), np.int8))
            elif kd == EV_RESTRICT:  # restrict_task -> set_restrictions({key: {worker}})
                eng.update_restrictions([t], [[w]], [1])
            elif kd == EV_RETIRE_REPLICA:  # remove_worker drops the retiring worker's replicas (:5263-5265)
                eng.remove_replicas([t], [w])
            elif kd == EV_RETIRE:  # then the worker itself, no transition: no resync
                eng.remove_worker(w)
            elif kd == EV_LOSE_WORKER:  # the whole remove_worker stimulus on the device
                lst = ht[hp[i]:hp[i + 1]]
                npr = int(x[i])
                assert eng.lose_worker(w, lst[:npr], lst[npr:], loss_order_rows(z, i),
                                       loss_killed(z, i, lst[:npr])) is not None, (i, eng.refusal)
            elif kd == EV_ERRED_RETRY:  # a retry / stale run: the reschedule's transitions on the device
                assert eng.reschedule(t) is not None, (i, eng.refusal)
            elif kd == EV_REFILL:  # handle_task_erred's queue refill (dgp_release_tasks of nothing)
                eng.release_tasks(np.zeros(0, np.int32), np.zeros(0, np.uint8))
            elif kd == EV_RESCHEDULE and device_resched and eng.reschedule(t) is not None:
                n_sync += 1  # decided on the device (dgp_reschedule): the fixture's resync rows unused
            elif kd == EV_RELEASE_KEYS and device_release:
                rp = z["rk_evptr"]  # the release's closure (loss.release_plan in the generator)
                rows = slice(rp[i], rp[i + 1])
                if release_states is not None:  # the engine states the release starts from
                    release_states.extend(eng.task_states()[z["rk_task"][rows]].tolist())
                assert eng.release_tasks(z["rk_task"][rows], z["rk_forget"][rows]) is not None, (i, eng.refusal)
                n_sync += 1
            elif kd in (EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS):
                # the scheduler decided this stimulus itself: its placements, then its state
                n = int(exp["stim_nplaced"][len(stim)])
                sl = slice(n0, n0 + n)
                eng.sync_placements(exp["pl_task"][sl], exp["pl_worker"][sl], exp["pl_comm"][sl], exp["pl_start"][sl],
                                    exp["pl_wsnbytes"][sl], exp["pl_route"][sl])
                if kd == EV_REMOVE_WORKER:
                    eng.remove_worker(w)
                d = sync_dump(z, n_sync)
                n_sync += 1
                eng.sync(None, d["tasks"], d["workers"], d["globals"])
            else:
                raise AssertionError(kd)
            stim.append(eng.num_placements() - n0)
        eng.snapshot()
    return np.array(stim, np.int32)


@pytest.mark.parametrize("name", svc_event_files())
def test_service_events_match_reference(name):
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    assert set(np.unique(z["ev_kind"]).tolist()) == set(range(8))  # every event kind is exercised
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        stim = drive_events(eng, g, z, exp)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


def test_service_events_refuse_what_they_do_not_model():
    """The last replica going, a paused worker taking a new graph, an erred cascade that
    would cancel work: refused (DGP_E_DEVICE / DGP_E_STATE), so the extension hands
    placement back instead of diverging."""
    from distributed_amd import _lib, graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(2000, 32, seed=5)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, results=False)
        eng.update_graph()
        p = eng.placements(0, 1)
        t, w = int(p["pl_task"][0]), int(p["pl_worker"][0])
        st, _ = eng.tasks_finished([t], [w], [0], [100], [0.0], [0.01])
        assert st.tolist() == [0]
        with pytest.raises(_lib.DgpError, match="does not model"):
            eng.remove_replicas([t], [w])  # its only replica
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, results=False)
        eng.update_graph()
        eng.set_worker_status(3, 0)
        h = dict(g2 := graphs.random_dag(200, 32, seed=6), prefix_default_dur=g["prefix_default_dur"],
                 group_prefix=g["group_prefix"])
        with pytest.raises(_lib.DgpError, match="paused"):
            eng.add_graph(dict(h, prio=g2["prio"] + len(g["prio"]), group_id=g2["group_id"] + len(g["group_prefix"]),
                               group_prefix=np.concatenate([g["group_prefix"], g2["group_prefix"]])))


@pytest.mark.parametrize("name", svc_retire_files())
def test_service_retiring_workers_match_reference(name):
    """Drained workers retire (Scheduler.remove_worker, scheduler.py:5180-5360, of a paused
    worker with nothing processing whose sole replicas were first copied elsewhere by
    add-keys, as retire_workers does): remove_worker runs no transition, so the engine
    follows it on the device -- its replicas dropped (dgp_remove_replicas), the worker
    removed (dgp_remove_worker) -- with no resync; every later placement, the snapshots and
    the final states equal the reference's."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    kinds = set(np.unique(z["ev_kind"]).tolist())
    assert {EV_RETIRE, EV_RETIRE_REPLICA} <= kinds and not kinds & {EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS}
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        stim = drive_events(eng, g, z, exp)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("name", svc_loss_files())
def test_service_worker_loss_on_the_engine(name):
    """Workers lost with processing tasks and sole replicas (Scheduler.remove_worker,
    scheduler.py:5180-5303: processing tasks released and re-placed, lost results
    recomputed, their processing dependents released to wait for them), decided by the
    engine (dgp_lose_worker) with no resync, interleaved with every modelled event: the
    placements each loss made, every later decision, the snapshots and the final states
    equal the reference's. svcwl_chain_*: the lost results recompute released dependencies
    in turn (recompute chains, in the scheduler's set orders: dgp_lose_worker_ordered).
    svcwl_killed_*: allowed_failures 1, so a task on its second lost worker errs at once
    (KilledWorker) with its waiting dependents."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    kinds = set(np.unique(z["ev_kind"]).tolist())
    assert EV_LOSE_WORKER in kinds and not kinds & {EV_REMOVE_WORKER, EV_RESCHEDULE, EV_RELEASE_KEYS}
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        stim = drive_events(eng, g, z, exp)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert len(out["pl_task"]) > g["n_tasks"]  # re-placements and recomputes: the logs grew
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("name", svc_resync_files())
@pytest.mark.parametrize("device_resched", [False, True], ids=["resync", "resched-on-device"])
def test_service_resync_matches_reference(name, device_resched):
    """Worker removal (Scheduler.remove_worker, scheduler.py:5180-5360: processing tasks
    released and re-placed, lost results recomputed), rescheduling (:7900-7927) and client
    releases (:5417-5430) decided by the scheduler itself, the engine resynchronised from
    its state (dgp_remove_worker, dgp_sync_*) after each, interleaved with every modelled
    event: the engine's own decisions from then on, the snapshots and the final states equal
    the reference's. resched-on-device: each reschedule decided by the engine instead
    (dgp_reschedule: released, waiting again, decide_worker), the scheduler's stimulus and
    resync only when it refuses (a task nobody needs)."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    assert set(np.unique(z["ev_kind"]).tolist()) == set(range(11))
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        stim = drive_events(eng, g, z, exp, device_resched=device_resched)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert len(out["pl_task"]) > g["n_tasks"]  # re-placements: the logs grew
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    # a forgotten task (client released, :2853) leaves SchedulerState.tasks; its engine row
    # stays, released (distributed_amd/sync.py)
    assert np.array_equal(out["final_state"], np.where(exp["final_state"] == 7, 0, exp["final_state"]))


@pytest.mark.parametrize("device_release", [False, True], ids=["resync", "release-on-device"])
@pytest.mark.parametrize("name", svc_release_files())
def test_service_client_releases(name, device_release):
    """Clients release wanted tasks (client-releases-keys, scheduler.py:5417-5430): results in
    memory (svcrel_*) and work in any state (svccan_*: waiting, processing, queued, no-worker
    cancelled, what they release and forget in turn) -- the keys forgotten or released, the
    dependencies nobody needs any more released or forgotten (_propagate_released :3337-3357,
    _propagate_forgotten :3359-3398), then the queue refill -- on the device
    (dgp_release_tasks, in the order loss.release_plan gives) or, for comparison, decided by
    the scheduler and resynchronised. Every placement, snapshot and final state equals the
    reference's (a forgotten task's row stays, released)."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    assert EV_RELEASE_KEYS in set(np.unique(z["ev_kind"]).tolist())
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        seen = [] if device_release else None
        stim = drive_events(eng, g, z, exp, device_release=device_release, release_states=seen)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    fe = np.where(exp["final_state"] == 7, 0, exp["final_state"])
    bad = np.nonzero(out["final_state"] != fe)[0]
    assert len(bad) == 0, (bad[:10], out["final_state"][bad[:10]], exp["final_state"][bad[:10]])
    if device_release and name.startswith("svccan_"):  # cancelled work of every kind, on the device
        cnt = np.bincount(np.array(seen, np.int64), minlength=6)
        print(name, "release ops by engine state (released, waiting, processing, queued, no-worker, memory):",
              cnt[:6].tolist())
        assert cnt[1] > 0 and cnt[2] > 0 and cnt[5] > 0, cnt


@pytest.mark.parametrize("name", svc_retry_files())
def test_service_erred_retries(name):
    """task-erred reports that do not err (stimulus_task_erred, scheduler.py:5111-5118): a
    retry (retries left: processing -> waiting through released) or a stale run's report from
    the worker the task runs on (processing -> released, re-waited) of a task something needs,
    re-placed on the device (dgp_reschedule), then handle_task_erred's queue refill (:5805,
    dgp_release_tasks of nothing). Every placement, snapshot and final state equals the
    reference's."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    kinds = set(np.unique(z["ev_kind"]).tolist())
    assert {EV_ERRED_RETRY, EV_REFILL} <= kinds
    assert {0.0, 1.0} <= set(z["ev_x"][z["ev_kind"] == EV_ERRED_RETRY].tolist())  # retries and stale runs
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        stim = drive_events(eng, g, z, exp)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("name", svc_p2p_files())
@pytest.mark.parametrize("device_resched", [False, True], ids=["resync", "resched-on-device"])
def test_service_p2p_shuffle_lifecycle_matches_reference(name, device_resched):
    """The P2P shuffle's scheduler-side lifecycle (gen_service.py p2p): the unpacks' _rootish
    set False when the first transfer runs (dgp_set_rootish), the barrier's completion
    placing them on the device as non-rootish, each unpack's restrict_task (dgp_update_
    restrictions) and Reschedule (the scheduler's stimulus, then dgp_sync_*; resched-on-device:
    dgp_reschedule, no resync), the re-placed unpacks completing: every placement, snapshot
    and final state equals the reference's ShuffleSchedulerPlugin-driven scheduler."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    assert {EV_SHUFFLE_INIT, EV_RESTRICT, EV_RESCHEDULE} <= set(np.unique(z["ev_kind"]).tolist())
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        stim = drive_events(eng, g, z, exp, device_resched=device_resched)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert np.array_equal(stim, exp["stim_nplaced"]), np.nonzero(stim != exp["stim_nplaced"])[0][:5]
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("name", svc_dep_graph_files() + svc_restr_graph_files() + svc_prio_graph_files())
def test_service_dependent_later_graph_matches_reference(name):
    """A later graph whose tasks depend on earlier ones (in memory, processing, waiting or
    queued when it arrives): dgp_add_graph appends it (the earlier tasks' dependents rows
    grow) without placing; the scheduler decides that update_graph stimulus (its placements
    and state are the fixture's, gen_service.py svcgdep_*) and the engine resyncs; every later
    placement, the snapshots and the final states are the engine's and equal the reference's."""
    from distributed_amd import _lib
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    at = int(z["g2_msg"])
    g2 = second_graph(g, z)
    restr = "g2_restr_flags" in z.files  # svcgrst_*: worker restrictions on the later graph
    rerank = "g2_prio_all" in z.files  # svcgprio_*: a user priority above the earlier tasks'
    assert restr or rerank or (np.asarray(g2["dep_idx"]) < 0).sum() > 0
    joins = {}
    for m, nt in zip(z["add_msg"].tolist() if "add_msg" in z.files else [],
                     z["add_nthreads"].tolist() if "add_nthreads" in z.files else []):
        joins.setdefault(m, []).append(nt)
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        for k in range(len(ptr) - 1):
            for i in range(ptr[k], ptr[k + 1]):
                for nt in joins.get(i, ()):
                    eng.add_worker(nt)
                if i == at:
                    n0 = eng.num_placements()
                    assert eng.add_graph(g2, defer=restr or rerank) == 0 and eng.num_placements() == n0
                    if rerank:  # every task's rank in the merged order (dgp_set_priorities)
                        eng.set_priorities(z["g2_prio_all"])
                    with pytest.raises(_lib.DgpError, match="dgp_sync"):  # nothing runs before the resync
                        eng.tasks_finished(*[[c] for c in msgs[i]])
                    sl = slice(n0, n0 + int(z["g2_nplaced"]))
                    eng.sync_placements(exp["pl_task"][sl], exp["pl_worker"][sl], exp["pl_comm"][sl],
                                        exp["pl_start"][sl], exp["pl_wsnbytes"][sl], exp["pl_route"][sl])
                    d = sync_dump(z, 0)
                    eng.sync(None, d["tasks"], d["workers"], d["globals"])
                    if restr:  # the new tasks' valid workers (dgp_update_restrictions)
                        rp, ri, rf = z["g2_restr_ptr"], z["g2_restr_idx"], z["g2_restr_flags"]
                        ts = np.flatnonzero(rf & 1)
                        w0 = eng.get_window()
                        eng.update_restrictions(g["n_tasks"] + ts, [ri[rp[t]:rp[t + 1]] for t in ts], rf[ts])
                        # the first restricted graph moves an "auto" engine to the 64-slot build
                        assert (w0, eng.get_window()) == (eng.auto_window(g), 64)
                st, _ = eng.tasks_finished(*[[c] for c in msgs[i]])
                assert st.tolist() == [0], (i, st)
            if ptr[k + 1] > ptr[k]:
                eng.snapshot()
        assert eng.n_tasks == g["n_tasks"] + len(g2["prio"])
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", svc_dep_graph_files() + svc_restr_graph_files() + svc_prio_graph_files())
def test_later_graph_stimulus_on_the_engine(name, per_message):
    """The same later graphs with their update_graph stimulus decided by the engine
    (dgp_graph_stimulus): appended deferred, the new tasks' valid workers
    (dgp_update_restrictions) or every task's merged rank (dgp_set_priorities) first, then
    the stimulus on the device -- the earlier tasks gain the new ones as waiters, the new ones
    wait on the earlier ones not in memory, the runnable ones go to processing / queued in
    priority order. svcgrec_*: some earlier dependencies are released and recomputed by that
    stimulus (recompute chains through the recommendation machine, in the scheduler's set
    orders: dgp_graph_stimulus_ordered). Its placements and every later one, the snapshots and
    the final states equal the reference's; no resync."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    at = int(z["g2_msg"])
    g2 = second_graph(g, z)
    restr = "g2_restr_flags" in z.files
    rerank = "g2_prio_all" in z.files
    joins = {}
    for m, nt in zip(z["add_msg"].tolist() if "add_msg" in z.files else [],
                     z["add_nthreads"].tolist() if "add_nthreads" in z.files else []):
        joins.setdefault(m, []).append(nt)
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        for k in range(len(ptr) - 1):
            i, e = ptr[k], ptr[k + 1]
            while i < e:
                for nt in joins.get(i, ()):
                    eng.add_worker(nt)
                if i == at:
                    n0 = eng.num_placements()
                    assert eng.add_graph(g2, defer=True) == 0 and eng.num_placements() == n0
                    if rerank:
                        eng.set_priorities(z["g2_prio_all"])
                    if restr:
                        rp, ri, rf = z["g2_restr_ptr"], z["g2_restr_idx"], z["g2_restr_flags"]
                        ts = np.flatnonzero(rf & 1)
                        eng.update_restrictions(g["n_tasks"] + ts, [ri[rp[t]:rp[t + 1]] for t in ts], rf[ts])
                    newp = eng.graph_stimulus(graph_order_rows(z))
                    assert newp == int(z["g2_nplaced"]) and eng.num_placements() == n0 + newp, (newp, z["g2_nplaced"])
                j = i + 1
                if not per_message:
                    while j < e and j not in joins and j != at:
                        j += 1
                st, _ = eng.tasks_finished(*(np.array(c) for c in zip(*msgs[i:j])))
                assert (st == 0).all(), (i, st)
                i = j
            if e > ptr[k]:
                eng.snapshot()
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("resident", [False, True], ids=["launch", "resident"])
@pytest.mark.parametrize("name", svc_event_files())
def test_task_messages_follow_replicas(name, resident):
    """dgp_task_messages (the who_has / nbytes fields of _task_to_msg, scheduler.py
    :3421-3450) after every event of a svcev_* stream, for the placements that event made:
    each dependency's who_has equals a model of SchedulerState.who_has driven by the same
    stream (the completing worker, then add-keys adding and release-worker-data removing
    replicas), in ascending worker order, and its nbytes the size its task-finished reported."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    kind, task, worker = z["ev_kind"], z["ev_task"], z["ev_worker"]
    hp, ht, hd = z["hb_ptr"], z["hb_task"], z["hb_dur"]
    dp, di = g["dep_ptr"], g["dep_idx"]
    who, nbytes = {}, {}
    checked = multi = pinned = 0
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, results=False)
        if resident:  # the task-finished answers carry the message fields (dgp_set_task_messages)
            eng.set_resident(True)
            eng.set_task_messages(True)
        eng.update_graph()
        for i in range(len(kind)):
            n0 = eng.num_placements()
            kd, t, w = int(kind[i]), int(task[i]), int(worker[i])
            if kd == EV_FINISHED:
                st, _ = eng.tasks_finished([t], [w], [int(z["ev_runid"][i])], [int(z["ev_nbytes"][i])],
                                           [float(z["ev_start"][i])], [float(z["ev_stop"][i])])
                assert st.tolist() == [0]
                who[t] = {w}
                nbytes[t] = int(z["ev_nbytes"][i])
            elif kd == EV_ADD_KEYS:
                eng.add_replicas([t], [w])
                who.setdefault(t, set()).add(w)
            elif kd == EV_RELEASE_DATA:
                eng.remove_replicas([t], [w])
                who[t].discard(w)
            elif kd in (EV_PAUSE, EV_RESUME):
                eng.set_worker_status(w, 1 if kd == EV_RESUME else 0)
            elif kd == EV_LONG_RUNNING:
                eng.long_running(t, float(z["ev_x"][i]))
            elif kd == EV_HEARTBEAT:
                ts = ht[hp[i]:hp[i + 1]]
                eng.heartbeat(float(z["ev_x"][i]), g["prefix_id"][ts], hd[hp[i]:hp[i + 1]])
            elif kd == EV_ERRED:
                eng.task_erred(t)
            elif kd == EV_SHUFFLE_INIT:  # _ensure_output_tasks_are_non_rootish: the unpacks' _rootish False
                ts = ht[hp[i]:hp[i + 1]]
                eng.set_rootish(ts, np.zeros(len(ts), np.int8))
            elif kd == EV_RESTRICT:  # restrict_task -> set_restrictions({key: {worker}})
                eng.update_restrictions([t], [[w]], [1])
            n1 = eng.num_placements()
            if n1 == n0:
                continue
            m = eng.task_messages(n0, n1 - n0)
            pl = eng.placements(n0, n1 - n0, columns=("pl_task", "pl_worker"))  # (the mailbox, resident)
            for j, x in enumerate(pl["pl_task"].tolist()):
                deps = di[dp[x]:dp[x + 1]].tolist()
                a, b = int(m["dep_ptr"][j]), int(m["dep_ptr"][j + 1])
                assert m["dep_task"][a:b].tolist() == deps, (i, x)
                # the reference's own message for this placement (gen_service.py records
                # _task_to_msg's who_has / nbytes per placement after update_graph)
                r = n0 + j - int(z["tm_first"])
                if r >= 0:
                    assert int(z["tm_task"][r]) == x, (i, x)
                    ra = int(z["tm_dep_ptr"][r])
                    assert z["tm_dep_task"][ra:ra + b - a].tolist() == deps
                for k, d in zip(range(a, b), deps):
                    hs = m["holder_idx"][m["holder_ptr"][k]:m["holder_ptr"][k + 1]].tolist()
                    assert hs == sorted(who[d]), (i, x, d, hs, who[d])
                    assert int(m["dep_nbytes"][k]) == nbytes[d], (i, x, d)
                    if r >= 0:
                        rk = ra + k - a
                        rh = z["tm_hold_idx"][z["tm_hold_ptr"][rk]:z["tm_hold_ptr"][rk + 1]].tolist()
                        assert hs == rh, (i, x, d, hs, rh)
                        assert int(m["dep_nbytes"][k]) == int(z["tm_dep_nbytes"][rk]), (i, x, d)
                        pinned += 1
                    multi += len(hs) > 1
                checked += 1
    assert checked > 1000 and multi > 0 and pinned > 1000, (checked, multi, pinned)


def svc_prefix_files():
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcpfx_") and f.endswith(".npz"))


def later_graph_of(z, k, pmax):
    """Later graph k of a svcpfx_* fixture over the engine-wide tables: priorities after every
    earlier task's, its prefix ids the engine's slots, its groups after the earlier ones."""
    p = f"g{k}_"
    return dict(dep_ptr=z[p + "dep_ptr"], dep_idx=z[p + "dep_idx"], prio=z[p + "prio"] + pmax + 1,
                prefix_id=z[p + "prefix_id"], group_id=z[p + "group_id"], wanted=z[p + "wanted"],
                rootish_override=z[p + "rootish_override"], prefix_default_dur=z[p + "defaults"],
                group_prefix=np.zeros(int(z[p + "n_groups"]), np.int32))


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", svc_prefix_files())
def test_service_prefix_table_compacts(name, per_message):
    """A session meeting more task prefixes than the engine's table (svcpfx_*: six later
    graphs with prefixes of their own, 75 over the stream): where a graph would not fit, the
    table is compacted to the live prefixes (dgp_remap_prefixes with every earlier task's slot,
    then the workers' and global rows in the new numbering, distributed_amd/prefixes.py run on
    the reference state), then the graph goes in (dgp_add_graph). Every placement, the
    per-round snapshots and the final task states equal the reference's."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    K = int(z["gk_n"])
    assert int(z["gk_prefix_names_total"]) > 64
    at = {int(z[f"g{k}_msg"]): k for k in range(K)}
    R = len(exp["round_nplaced"]) + 2
    status, remaps = [], 0
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        pmax = int(np.max(g["prio"]))
        for kk in range(len(ptr) - 1):
            i, e = ptr[kk], ptr[kk + 1]
            while i < e:  # batches end at each submission
                if i in at:
                    k = at[i]
                    if f"g{k}_remap_slots" in z.files:
                        d = sync_dump(z, int(z[f"g{k}_remap_dump"]))
                        eng.remap_prefixes(z[f"g{k}_remap_slots"], z[f"g{k}_remap_defaults"])
                        eng.sync(None, None, d["workers"], d["globals"])
                        remaps += 1
                    gk = later_graph_of(z, k, pmax)
                    pmax = int(gk["prio"].max())
                    n0 = eng.num_placements()
                    newp = eng.add_graph(gk)
                    assert newp == int(z[f"g{k}_nplaced"]) and eng.num_placements() == n0 + newp
                j = i + 1
                if not per_message:
                    while j < e and j not in at:
                        j += 1
                t, w, r, nb, a, b = (np.array(c) for c in zip(*msgs[i:j]))
                st, _ = eng.tasks_finished(t, w, r, nb, a, b)
                status.extend(st.tolist())
                i = j
            if e > ptr[kk]:
                eng.snapshot()
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert remaps >= 3
    assert (np.array(status) == 0).all()
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])
