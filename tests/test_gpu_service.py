"""Service mode (needs an MI355X): the engine driven the way a live scheduler drives it,
one task-finished message (or one batch) per ``dgp_tasks_finished`` call, with the device
state resident between calls.

* every golden fixture is replayed through the service entry one completion at a time and
  one round per call: the placement log, the per-round snapshots (taken with
  ``dgp_snapshot`` at the round boundaries) and the final task states equal the
  reference's, bit for bit;
* the ``svc_*`` fixtures (``tests/golden/gen_service.py``) carry the reference's own answers
  (``Scheduler.stimulus_task_finished``, distributed/scheduler.py:5025-5092) to a message
  stream that mixes stale, duplicate, already-in-memory, forgotten-key and unknown-worker
  reports into the completions: the engine's status per message must equal them, and the
  placements must be unaffected;
* the ``svcaddw_*`` fixtures have workers join mid-stream (Scheduler.add_worker,
  distributed/scheduler.py:4308-4441): each goes to ``dgp_add_worker`` before the message it
  preceded in the reference, and the queue refill it makes, the later placements, the
  snapshots (as wide as the final worker count) and the task states must equal the reference's;
* the ``svcgraph_*`` fixtures submit a second, independent graph mid-stream
  (Scheduler.update_graph on a running scheduler, distributed/scheduler.py:4662-4751): it
  goes to ``dgp_add_graph`` before the message it preceded in the reference;
* the ``svc_steal_*`` fixtures interleave confirmed steals (WorkStealing.move_task_confirm,
  distributed/stealing.py:376-384) with that stream: each goes to ``dgp_move_task`` before
  the message it preceded in the reference, and the placements, snapshots and statuses
  that follow must still equal the reference's.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files, second_graph, svc_add_worker_files, svc_second_graph_files, svc_steal_files
from oracle import oracle
from test_gpu_parity import PL_KEYS, ROUND_KEYS, assert_same

pytestmark = pytest.mark.gpu


def fixture_messages(g, exp):
    """The genuine completions of the replay protocol, round by round (run_id order)."""
    nb, a, b = g["nbytes"], g["start"], g["stop"]
    msgs, ptr, pos = [], [0], 0
    for n in exp["round_nplaced"]:
        for r in range(pos, pos + int(n)):
            t = int(exp["pl_task"][r])
            msgs.append((t, int(exp["pl_worker"][r]), r, int(nb[t]), float(a[t]), float(b[t])))
        pos += int(n)
        ptr.append(len(msgs))
    return msgs, ptr


def drive(eng, msgs, ptr, per_message):
    """Feed the message stream; snapshot after each round. Returns the statuses."""
    status = []
    for k in range(len(ptr) - 1):
        chunk = msgs[ptr[k]:ptr[k + 1]]
        if not chunk:
            continue
        groups = [[m] for m in chunk] if per_message else [chunk]
        for grp in groups:
            t, w, r, nb, a, b = (np.array(c) for c in zip(*grp))
            st, _ = eng.tasks_finished(t, w, r, nb, a, b)
            status.extend(st.tolist())
        eng.snapshot()
    return np.array(status, np.int8)


def run_service(g, cfg, exp, msgs, ptr, per_message, resident=False):
    from distributed_amd.engine import PlacementEngine

    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.set_resident(resident)
        eng.update_graph()
        status = drive(eng, msgs, ptr, per_message)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    return out, status


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", golden_files())
def test_service_matches_reference_fixture(name, per_message):
    g, cfg, exp, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    msgs, ptr = fixture_messages(g, exp)
    out, status = run_service(g, cfg, exp, msgs, ptr, per_message)
    assert (status == 0).all(), np.bincount(status)
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


RESIDENT = ["c2var_sat1.1.npz", "c2mini_satinf.npz", "c3mini_sat1.1.npz", "restr_sat1.1.npz", "c2p12_sat1.1.npz",
            "svc_c2var_sat1.1.npz"]


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", RESIDENT)
def test_resident_service_matches_reference_fixture(name, per_message):
    """The same message streams through the resident kernel (dgp_set_resident): each batch
    goes through the pinned mailbox while the kernel stays launched; the snapshot between
    rounds ends it (every other entry point does) and the next batch launches it again."""
    g, cfg, exp, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    msgs, ptr = fixture_messages(g, exp)
    out, status = run_service(g, cfg, exp, msgs, ptr, per_message, resident=True)
    assert (status == 0).all(), np.bincount(status)
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("resident", [False, True], ids=["launch", "resident"])
@pytest.mark.parametrize("name", ["c2var_sat1.1.npz", "restr_sat1.1.npz", "c3mini_sat1.1.npz"])
def test_window_switched_between_calls(name, resident):
    """Both stream-kernel builds on ONE engine (dgp_set_window, ABI 19): the window alternates
    32 / 64 every call, so consecutive batches run on different builds over the same resident
    state; the placements, snapshots and final states still equal the reference's."""
    from distributed_amd.engine import PlacementEngine

    g, cfg, exp, meta = oracle.load_fixture(os.path.join(GOLDEN, name))
    msgs, ptr = fixture_messages(g, exp)
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.set_resident(resident)
        eng.update_graph()
        status, calls = [], 0
        for k in range(len(ptr) - 1):
            chunk = msgs[ptr[k]:ptr[k + 1]]
            if not chunk:
                continue
            for i in range(0, len(chunk), 7):  # batches of 7 messages
                eng.set_window(64 if calls % 2 else 32)
                assert eng.get_window() == (64 if calls % 2 else 32)
                t, w, r, nb, a, b = (np.array(c) for c in zip(*chunk[i:i + 7]))
                st, _ = eng.tasks_finished(t, w, r, nb, a, b)
                status.extend(st.tolist())
                calls += 1
            eng.snapshot()
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert calls > 10
    assert (np.array(status) == 0).all()
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


SVC = sorted(f for f in golden_files() if f.startswith("svc_"))


@pytest.mark.parametrize("resident", [False, True], ids=["launch", "resident"])
@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", SVC)
def test_service_stale_duplicate_memory(name, per_message, resident):
    """The reference's answers to stale / duplicate / in-memory / unknown reports (also through
    the resident kernel, whose answers split a batch into segments exactly as k_svc_append)."""
    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    out, status = run_service(g, cfg, exp, msgs, ptr, per_message, resident)
    want = z["msg_status"]
    bad = np.nonzero(status != want)[0]
    assert len(bad) == 0, f"{len(bad)} status mismatches, first message {bad[0]}: {status[bad[0]]} vs {want[bad[0]]}"
    assert set(np.unique(want).tolist()) >= {0, 1, 2, 3, 4}  # every answer class is exercised
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


def drive_posted(eng, msgs, ptr):
    """``drive`` one message per dgp_tasks_finished_post / _wait (GPUPlacementExtension's
    overlapped path): the entry points that touch the device refuse while a batch is posted,
    and each answer's new placements and message fields through ``engine.answer`` equal
    placements() + task_messages() of the same range."""
    from distributed_amd import _lib

    status, n, refused = [], eng.num_placements(), 0
    for k in range(len(ptr) - 1):
        chunk = msgs[ptr[k]:ptr[k + 1]]
        if not chunk:
            continue
        for m in chunk:
            eng.tasks_finished_post(*[(x,) for x in m])
            if refused < 2:  # the kernel is inside the request: no other call meanwhile
                with pytest.raises(_lib.DgpError, match="posted"):
                    eng.num_placements() if refused == 0 else eng.placements(0, 1)
                refused += 1
            st, new = eng.tasks_finished_wait()
            status.extend(st.tolist())
            if new:
                tasks, workers, fields = eng.answer(n, new, True)
                p = eng.placements(n, new, columns=("pl_task", "pl_worker"))
                tm = eng.task_messages(n, new)
                assert tasks == p["pl_task"].tolist() and workers == p["pl_worker"].tolist()
                for got, key in zip(fields, ("dep_ptr", "dep_task", "dep_nbytes", "holder_ptr", "holder_idx")):
                    assert got == tm[key].tolist(), key
                n += new
        eng.snapshot()
    return np.array(status, np.int8)


@pytest.mark.parametrize("resident", [False, True], ids=["launch", "resident"])
@pytest.mark.parametrize("name", ["c2var_sat1.1.npz", "c3mini_sat1.1.npz", "svc_c2var_sat1.1.npz"])
def test_posted_service_matches_reference_fixture(name, resident):
    """dgp_tasks_finished_post / _wait (ABI 15) give what dgp_tasks_finished gives: the
    reference's statuses, placements, snapshots and final states, launch per call and
    through the resident kernel (with the mailbox's message fields)."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    if name.startswith("svc_"):
        z = np.load(path, allow_pickle=False)
        msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                        z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
        ptr, want = z["msg_round_ptr"].tolist(), z["msg_status"]
    else:
        msgs, ptr = fixture_messages(g, exp)
        want = np.zeros(len(msgs), np.int8)
    R = len(exp["round_nplaced"]) + 2
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.set_resident(resident)
        eng.set_task_messages(resident)
        eng.update_graph()
        status = drive_posted(eng, msgs, ptr)
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert np.array_equal(status, want)
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


def test_posted_batch_guards():
    """A wait with nothing posted and a second post are refused; closing the engine with a
    batch posted waits for its answer."""
    from distributed_amd import _lib, graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(2000, 32, seed=3)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    for resident in (False, True):
        eng = PlacementEngine(0)
        eng.load(g, cfg)
        eng.set_resident(resident)
        eng.update_graph()
        with pytest.raises(_lib.DgpError, match="no batch posted"):
            eng.tasks_finished_wait()
        p = eng.placements(0, 2)
        eng.tasks_finished_post(p["pl_task"][:1], p["pl_worker"][:1], [0], [100], [0.0], [0.01])
        with pytest.raises(_lib.DgpError, match="posted"):
            eng.tasks_finished_post(p["pl_task"][1:], p["pl_worker"][1:], [1], [100], [0.0], [0.01])
        with pytest.raises(_lib.DgpError, match="posted"):
            eng.tasks_finished(p["pl_task"][1:], p["pl_worker"][1:], [1], [100], [0.0], [0.01])
        st, _ = eng.tasks_finished_wait()
        assert st.tolist() == [0]
        eng.tasks_finished_post(p["pl_task"][1:], p["pl_worker"][1:], [1], [100], [0.0], [0.01])
        eng.close()  # waits for the posted answer first


def test_service_empty_batch_and_mode_guard():
    """An empty batch is a no-op; a replay cannot continue a service-mode engine."""
    from distributed_amd import _lib, graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(2000, 32, seed=3)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    with PlacementEngine(0) as eng:
        eng.load(g, cfg)
        eng.update_graph()
        st, newp = eng.tasks_finished([], [], [])
        assert len(st) == 0 and newp == 0
        p = eng.placements(0, 1)
        st, newp = eng.tasks_finished(p["pl_task"], p["pl_worker"], [0], [100], [0.0], [0.01])
        assert st.tolist() == [0]
        with pytest.raises(_lib.DgpError):
            eng.run_rounds(-1)


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", svc_steal_files())
def test_service_with_confirmed_steals(name, per_message):
    """Steal confirmations on the device between task-finished messages."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    steal_at = {}
    for i, t, h in zip(z["steal_msg"].tolist(), z["steal_task"].tolist(), z["steal_thief"].tolist()):
        steal_at.setdefault(i, []).append((t, h))
    assert len(z["steal_task"]) > 50
    R = len(exp["round_nplaced"]) + 2
    status = []
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        for k in range(len(ptr) - 1):
            i, e = ptr[k], ptr[k + 1]
            while i < e:  # batches end at the next steal (per message: one message each)
                for t, h in steal_at.get(i, ()):
                    eng.move_task(t, h)
                j = i + 1
                if not per_message:
                    while j < e and j not in steal_at:
                        j += 1
                t, w, r, nb, a, b = (np.array(c) for c in zip(*msgs[i:j]))
                st, _ = eng.tasks_finished(t, w, r, nb, a, b)
                status.extend(st.tolist())
                i = j
            if e > ptr[k]:
                eng.snapshot()
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    status = np.array(status, np.int8)
    want = z["msg_status"]
    bad = np.nonzero(status != want)[0]
    assert len(bad) == 0, f"{len(bad)} status mismatches, first message {bad[0]}: {status[bad[0]]} vs {want[bad[0]]}"
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


def test_move_task_rejects_a_task_not_processing():
    from distributed_amd import _lib, graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(2000, 32, seed=3)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, results=False)
        eng.update_graph()
        placed = set(eng.placements()["pl_task"].tolist())
        waiting = next(t for t in range(g["n_tasks"]) if t not in placed)
        with pytest.raises(_lib.DgpError):
            eng.move_task(waiting, 0)


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", svc_add_worker_files())
def test_service_with_workers_joining(name, per_message):
    """Workers join a running engine (dgp_add_worker_at) between task-finished messages; in
    the svcaddw_order_* fixtures at addresses that sort among the known ones (every later
    worker's index moves up on the device) and some of them paused, resuming later."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    add_at = {}  # message index -> the joins before it: (nthreads, position, running)
    n_add = len(z["add_nthreads"])
    pos = z["add_pos"].tolist() if "add_pos" in z else [None] * n_add
    run = z["add_running"].tolist() if "add_running" in z else [1] * n_add
    for i, nt, p_, r_ in zip(z["add_msg"].tolist(), z["add_nthreads"].tolist(), pos, run):
        add_at.setdefault(i, []).append((nt, p_, r_))
    for i, w in zip(*((z["res_msg"].tolist(), z["res_worker"].tolist()) if "res_msg" in z else ((), ()))):
        add_at.setdefault(i, []).append((0, w, 2))  # a paused joiner resumes (worker-status-change)
    W0 = len(g["nthreads"])
    R = len(exp["round_nplaced"]) + 2
    status, refill = [], 0
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        for k in range(len(ptr) - 1):
            i, e = ptr[k], ptr[k + 1]
            while i < e:  # batches end at the next worker addition
                for nt, p_, r_ in add_at.get(i, ()):
                    n0 = eng.num_placements()
                    if r_ == 2:
                        newp = eng.set_worker_status(p_, 1)
                    else:
                        newp = eng.add_worker(nt, running=bool(r_), position=p_)
                    assert eng.num_placements() == n0 + newp
                    refill += newp
                j = i + 1
                if not per_message:
                    while j < e and j not in add_at:
                        j += 1
                t, w, r, nb, a, b = (np.array(c) for c in zip(*msgs[i:j]))
                st, _ = eng.tasks_finished(t, w, r, nb, a, b)
                status.extend(st.tolist())
                i = j
            if e > ptr[k]:
                eng.snapshot()
        assert eng.n_workers == W0 + len(z["add_nthreads"])
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert (np.array(status) == 0).all()
    if cfg["saturation"] != "inf":
        assert refill > 0  # the joins took queued tasks
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


@pytest.mark.parametrize("per_message", [True, False], ids=["per-message", "per-round"])
@pytest.mark.parametrize("name", svc_second_graph_files())
def test_service_with_a_second_graph(name, per_message):
    """A second graph submitted to a running engine (dgp_add_graph) between messages."""
    from distributed_amd.engine import PlacementEngine

    path = os.path.join(GOLDEN, name)
    g, cfg, exp, meta = oracle.load_fixture(path)
    z = np.load(path, allow_pickle=False)
    msgs = list(zip(z["msg_task"].tolist(), z["msg_worker"].tolist(), z["msg_runid"].tolist(),
                    z["msg_nbytes"].tolist(), z["msg_start"].tolist(), z["msg_stop"].tolist()))
    ptr = z["msg_round_ptr"].tolist()
    at = int(z["g2_msg"])
    g2 = second_graph(g, z)
    joins = {}  # workers joining in the same stream (svcgraph_joins_*): before the graph
    for m, nt in zip(z["add_msg"].tolist() if "add_msg" in z.files else [],
                     z["add_nthreads"].tolist() if "add_nthreads" in z.files else []):
        joins.setdefault(m, []).append(nt)
    R = len(exp["round_nplaced"]) + 2
    status = []
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, snapshots=R, results=False)
        eng.update_graph()
        for k in range(len(ptr) - 1):
            i, e = ptr[k], ptr[k + 1]
            while i < e:  # batches end at the submission and at each join
                for nt in joins.get(i, ()):
                    eng.add_worker(nt)
                if i == at:
                    n0 = eng.num_placements()
                    newp = eng.add_graph(g2)
                    assert eng.num_placements() == n0 + newp
                j = i + 1
                if not per_message:
                    while j < e and j != at and j not in joins:
                        j += 1
                t, w, r, nb, a, b = (np.array(c) for c in zip(*msgs[i:j]))
                st, _ = eng.tasks_finished(t, w, r, nb, a, b)
                status.extend(st.tolist())
                i = j
            if e > ptr[k]:
                eng.snapshot()
        assert eng.n_tasks == g["n_tasks"] + len(g2["prio"])
        out = eng.placements()
        out.update(eng.snapshots(R))
        out["final_state"] = eng.task_states()
    assert (np.array(status) == 0).all()
    assert_same(out, exp, PL_KEYS + ROUND_KEYS)
    assert np.array_equal(out["final_state"], exp["final_state"])


def test_joins_and_later_graphs_reject_what_they_do_not_model():
    """dgp_add_worker / dgp_add_graph answer with an error (the extension then hands
    placement back to the scheduler) instead of placing wrongly."""
    from distributed_amd import _lib, graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(2000, 32, seed=3)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    h = graphs.random_dag(500, 32, seed=4)
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, results=False)
        with pytest.raises(_lib.DgpError):  # before update_graph
            eng.add_worker(2)
        with pytest.raises(_lib.DgpError):
            eng.add_graph(dict(h, prio=h["prio"] + g["n_tasks"]))
        eng.update_graph()
        with pytest.raises(_lib.DgpError):  # nthreads out of range
            eng.add_worker(0)
        with pytest.raises(_lib.DgpError):  # priorities not after the first graph's
            eng.add_graph(h)
        dep_old = dict(h, prio=h["prio"] + g["n_tasks"], dep_idx=np.asarray(h["dep_idx"]) + 10_000)
        with pytest.raises(_lib.DgpError):  # a dependency outside the new graph
            eng.add_graph(dep_old)
        assert eng.add_worker(3) >= 0 and eng.n_workers == 33
        n1 = eng.num_placements()
        newp = eng.add_graph(dict(h, prio=h["prio"] + g["n_tasks"]))
        assert eng.num_placements() == n1 + newp
        assert eng.n_tasks == 2500
        st = eng.task_states()[2000:]  # every new task went waiting, queued or processing
        assert set(np.unique(st).tolist()) <= {1, 2, 3} and (st == 3).sum() + newp >= 50  # 50 roots
