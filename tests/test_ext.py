"""The drop-in Scheduler extension (distributed_amd/ext.py) inside the reference scheduler.

Runs ``tests/ext_driver.py`` under the image's python3.9 with the reference imported from
/root/reference (``tests/golden/_refshim.py``). Neither exists on the GPU box, so there
these tests skip; the engine side of the same message streams is covered on the GPU by
``tests/test_gpu_service.py`` (one dgp_tasks_finished call per message).
"""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

PY39 = "/opt/conda/bin/python3.9"
DRIVER = os.path.join(REPO, "tests", "ext_driver.py")
HAVE_REF = os.path.exists(PY39) and os.path.isdir("/root/reference/distributed")

pytestmark = pytest.mark.skipif(not HAVE_REF, reason="needs the reference + python3.9 (build container only)")

FIXTURES = ["c1_sat1.1.npz", "c1_satinf.npz", "c2var_sat1.1.npz", "c2var_sat2.5.npz", "c2var_satinf.npz",
            "c2p12_sat1.1.npz", "c3mini_sat1.1.npz", "nodep_w19_sat1.1.npz", "nodep_w20_satinf.npz",
            "nodep_w24_sat1.1.npz", "occupancy_comm.npz", "sat_factor_0.1.npz", "sat_factor_2.5.npz",
            "sat_factor_inf.npz", "restr_sat1.1.npz", "restr_satinf.npz", "restr_nodep_w24.npz",
            "restr_noworker_sat1.1.npz"]


def drive(names, *flags):
    env = dict(os.environ, PYTHONHASHSEED="0")
    env.pop("PYTHONPATH", None)
    out = subprocess.run([PY39, DRIVER, *flags, *names], capture_output=True, text=True, env=env, timeout=600,
                         cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    return [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]


def test_extension_places_every_task_from_the_engine():
    """Upload conversion, decision order, validate=True agreement and exact records."""
    res = drive(FIXTURES)
    assert [r["fixture"] for r in res] == FIXTURES
    for r in res:
        assert r["active"] and r["device_decisions"] == r["placements"], r
    assert next(r for r in res if r["fixture"] == "restr_noworker_sat1.1.npz")["device_no_worker"] > 0


def test_extension_ingests_a_200k_graph_in_bulk():
    """f4 ingestion (ext_driver.py --ingest): the extension's update_graph hook turns a 200k-task
    C2-shaped graph of reference TaskStates into the engine's arrays (checked against the
    graph they were built from). Correctness only: the wall-clock figure (about 2 us per task
    on this container) is reported, and goes to DESIGN §7 from a dedicated run; a shared CPU
    must not fail this test."""
    (r,) = drive(["200000"], "--ingest")
    assert r["n_tasks"] == 200000 and r["n_edges"] > 600000, r
    print(f"ingestion: {r['us_per_task']:.2f} us per task")


def test_extension_batches_and_synchronous_calls():
    """The other two ways the task-finished messages reach the engine: a comm.read batch of
    one worker's consecutive messages through handle_stream (one posted call for several
    messages, the answer taken at the first decision), and the engine call made
    synchronously before the handler (overlap off). Same decisions, validate=True."""
    names = ["c2var_sat1.1.npz", "c3mini_sat1.1.npz", "restr_sat1.1.npz", "nodep_w24_sat1.1.npz"]
    for flags in (("--stream",), ("--nooverlap",)):
        res = drive(names, *flags)
        assert [r["fixture"] for r in res] == names
        for r in res:
            assert r["active"] and r["device_decisions"] == r["placements"], (flags, r)
            if flags == ("--stream",):
                assert r["engine_calls"] == r["reads"] <= r["messages"], r
            else:
                assert r["us_overlap_window"] == 0.0, r


def test_ab_timing_harness():
    """ext_driver.py --ab (DESIGN §7's per-message A/B): both sides of one process make the
    reference's placements from the same messages, every placement on the extension's side
    comes from the engine, and the report carries the difference with its interval."""
    r = drive(["c2var_sat1.1.npz"], "--ab")[0]
    assert r["mode"] == "ab" and r["messages"] > 1000, r
    for k in ("reference_us_per_message", "extension_host_us_per_message", "diff_us_per_message", "diff_ci95_us"):
        assert isinstance(r[k], float) and r[k] == r[k], (k, r)


def test_extension_follows_workers_joining():
    """Scheduler.add_worker mid-stream: the plugin hook adds the worker to the engine, and
    the scheduler's queue refill takes the engine's decisions (validate=True agrees)."""
    names = ["svcaddw_c2var_sat1.1.npz", "svcaddw_c2mini_sat1.0.npz", "svcaddw_c2mini_satinf.npz",
             "svcaddw_restr_sat1.1.npz", "svcaddw_p16_sat1.1.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["device_decisions"] == r["placements"], r
        assert r["workers_added"] == r["joins"] > 0, r


def test_extension_follows_workers_joining_in_address_order():
    """Workers join at addresses that sort among the known ones (SortedDict order, scheduler.py
    :3746 / :4353) and some join paused, resuming later: the extension inserts each at its
    place (dgp_add_worker_at, every later index moves up) and stays active; every decision
    is the engine's and validate=True agrees."""
    names = ["svcaddw_order_sat1.1.npz", "svcaddw_order_satinf.npz"]
    res = drive(names)
    for r in res:
        assert r["active"] and r["device_decisions"] == r["placements"], r
        assert r["workers_added"] == r["joins"] > 0 and r["workers_inserted"] > 0, r
        assert r["workers_added_paused"] > 0 and r["resumes"] > 0, r


def test_extension_follows_a_second_graph():
    """A second, independent graph submitted to the running scheduler: the plugin hook
    appends it to the engine (dgp_add_graph); every decision still comes from the engine."""
    names = ["svcgraph_c2var_sat1.1.npz", "svcgraph_c2mini_satinf.npz", "svcgraph_joins_sat1.1.npz",
             "svcgraph_restr_sat1.1.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["device_decisions"] == r["placements"] and r["graphs"] == 2, r


LATER = ["svcgdep_c2mini_satinf.npz", "svcgdep_c2var_sat1.1.npz", "svcgdep_joins_sat1.0.npz",
         "svcgrst_c2var_sat1.1.npz", "svcgrst_dep_satinf.npz", "svcgprio_c2mini_satinf.npz", "svcgprio_c2var_sat1.1.npz",
         "svcgrec_c2var_sat1.1.npz", "svcgrec_c2mini_satinf.npz"]


def test_extension_runs_later_graph_stimuli_on_the_engine():
    """A later graph whose tasks depend on earlier ones (in memory, processing, waiting or
    queued), carry worker restrictions (scheduler.py:4908-4922) or outrank earlier tasks by a
    user priority (_set_priorities :4934-4981): the extension appends it (dgp_add_graph /
    _deferred), hands the engine the new tasks' valid workers (dgp_update_restrictions) or
    every task's merged rank (dgp_set_priorities), and the engine runs that update_graph
    stimulus itself (dgp_graph_stimulus): no resync, every decision the engine's
    (validate=True), the extension active."""
    res = drive(LATER)
    assert [r["fixture"] for r in res] == LATER
    for r in res:
        assert r["active"] and r["graphs"] == 2 and r["resyncs"] == 0, r
        assert r["graph_stimuli_on_device"] == 1 and r["device_decisions"] == r["placements"], r


def test_extension_resyncs_later_graphs_without_the_engine_stimulus():
    """The same streams with an engine that has no dgp_graph_stimulus (--resync): the
    scheduler decides that stimulus, the engine resyncs once from its state (the rows equal
    the reference dump, every new task and every earlier task it depends on among them) and
    every later decision is the engine's (validate=True). The path the extension keeps for an
    earlier dependency that is released, erred or forgotten."""
    res = drive(LATER, "--resync")
    for r in res:
        assert r["active"] and r["graphs"] == 2 and r["resyncs"] == 1, r
        assert r["device_decisions"] + r["host_placements"] == r["placements"], r


EVENTS = ["svcev_c2var_sat1.1.npz", "svcev_c2mini_satinf.npz", "svcev_dense_sat1.0.npz"]


def test_extension_follows_service_events():
    """add-keys, release-worker-data, worker pause / resume, long-running, heartbeats and
    task-erred through the scheduler's own handlers: the extension forwards each to its
    engine call with the arguments the reference state implies, stays active, and every
    placement (validate=True) is the reference's."""
    res = drive(EVENTS)
    assert [r["fixture"] for r in res] == EVENTS
    for r in res:
        assert r["active"] and r["device_decisions"] == r["placements"], r
        for op in ("add_replicas", "remove_replicas", "set_worker_status", "long_running", "heartbeat",
                   "task_erred"):
            assert r["calls"].get(op, 0) > 0, (op, r)


RESYNC = ["svcrs_c2var_sat1.1.npz", "svcrs_c2mini_satinf.npz"]
P2P = ["svcp2p_sat1.1.npz", "svcp2p_satinf.npz"]


def test_extension_follows_the_p2p_shuffle_lifecycle():
    """The P2P shuffle as a live scheduler runs it (gen_service.py p2p), the reference's own
    ShuffleSchedulerPlugin acting on the scheduler: when the first transfer runs,
    _ensure_output_tasks_are_non_rootish sets _rootish False on every unpack by attribute
    assignment (shuffle/_scheduler_plugin.py:150-151, :254-278) -- the extension's wrapper
    hands the new overrides to the engine (dgp_set_rootish); the barrier's completion places
    the unpacks on the device as non-rootish; each unpack's restrict_task -> set_restrictions
    (:101-115, :281-293 -> scheduler.py:7702-7707, the *method*) reaches the engine
    (dgp_update_restrictions); its Reschedule runs on the engine too (dgp_reschedule: the
    unpack released from its worker and placed again on its restriction). The extension stays
    active throughout with no resync; every placement is the engine's (validate=True)."""
    res = drive(P2P)
    assert [r["fixture"] for r in res] == P2P
    for r in res:
        assert r["active"] and r["resyncs"] == 0 and r["calls"]["reschedule"] > 0, r
        assert r["device_decisions"] == r["placements"], r


def test_extension_resyncs_after_stimuli_it_does_not_model():
    """Worker removal (Scheduler.remove_worker), rescheduling and client releases in the
    stream, with an engine that does not restate them (no lose_worker / reschedule /
    release_tasks): the plugin transition hook suspends the engine at the first transition it
    does not model, the scheduler decides that stimulus, and the extension resynchronises the
    engine (dgp_remove_worker, dgp_sync_*): the rows it sends cover every task whose state
    changed (checked against a full dump), the worker / global rows equal the fixture's
    dumps, the extension stays active and every other placement is the engine's
    (validate=True)."""
    res = drive(RESYNC, "--resync-only")
    assert [r["fixture"] for r in res] == RESYNC
    for r in res:
        assert r["active"] and r["resyncs"] > 0 and r["calls"].get("workers_lost_on_device", 0) == 0, r
        assert r["device_decisions"] + r["host_placements"] == r["placements"], r


def test_extension_decides_every_resync_stimulus_on_the_engine():
    """The same streams with the engine's worker-loss, reschedule and client-release
    operations: every one of those stimuli is restated on the engine (dgp_lose_worker_ordered,
    dgp_reschedule, dgp_release_tasks), no resync, every placement the engine's."""
    res = drive(RESYNC)
    assert [r["fixture"] for r in res] == RESYNC
    for r in res:
        assert r["active"] and r["resyncs"] == 0, r
        for op in ("workers_lost_on_device", "reschedule", "release_tasks"):
            assert r["calls"].get(op, 0) > 0, (op, r)
        assert r["device_decisions"] == r["placements"], r


def test_extension_follows_retiring_workers_on_the_device():
    """Drained workers retire (svcrt_*: paused, nothing processing, sole replicas copied
    elsewhere first): Scheduler.remove_worker runs no transition, so the extension drops the
    worker's replicas (dgp_remove_replicas through the replica hook) and removes it on the
    device (dgp_remove_worker) with no resync; every placement is the engine's
    (validate=True) and the extension stays active."""
    names = ["svcrt_c2var_sat1.1.npz", "svcrt_c2mini_satinf.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["resyncs"] == 0 and r["calls"]["workers_removed_on_device"] > 0, r
        assert r["device_decisions"] == r["placements"], r


def test_extension_runs_worker_losses_on_the_engine():
    """Workers lost with processing tasks and sole replicas (svcwl_*): the extension's
    remove_worker wrapper hands the whole stimulus to the engine (dgp_lose_worker, with the
    worker's processing tasks and replicas in the scheduler's own iteration order) before
    Scheduler.remove_worker runs; its transitions (processing tasks released and re-placed,
    lost results recomputed, their processing dependents released to wait) take the engine's
    decisions, validate=True re-derives each; no resync, every placement the engine's.
    svcwl_chain_*: lost results whose dependencies were released recompute them in turn; the
    extension passes the set orders the cascade follows (distributed_amd/loss.py), equal to
    the ones the fixture recorded. svcwl_killed_*: a task on its second lost worker errs at once
    (KilledWorker, allowed_failures 1), its waiting dependents with it."""
    names = ["svcwl_c2var_sat1.1.npz", "svcwl_c2mini_satinf.npz", "svcwl_chain_c2var_sat1.1.npz",
             "svcwl_chain_c2mini_satinf.npz", "svcwl_killed_c2var_sat1.1.npz", "svcwl_killed_c2mini_satinf.npz",
             "svcwl_killed0_c2var_sat1.1.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["resyncs"] == 0 and r["calls"]["workers_lost_on_device"] >= 10, r
        assert r["device_decisions"] == r["placements"], r


def test_extension_follows_client_releases_on_the_engine():
    """Clients release results in memory (svcrel_*) and cancel wanted work in any state
    (svccan_*): the extension computes what the scheduler's transitions will reach, in their
    order (loss.release_plan: the keys released or forgotten, the work and results released
    and forgotten with them) and the engine follows on the device (dgp_release_tasks) before
    the handler runs; the closures equal the generator's, no resync, every placement the
    engine's (validate=True)."""
    names = ["svcrel_c2var_sat1.1.npz", "svcrel_c2mini_satinf.npz", "svccan_c2var_sat1.1.npz",
             "svccan_c2mini_satinf.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["resyncs"] == 0 and r["calls"]["release_tasks"] >= 50, r
        assert r["device_decisions"] == r["placements"], r
        if r["fixture"].startswith("svccan_"):  # wanted leaves cancelled through cancel-keys
            assert r["cancels"] > 0, r


def test_extension_follows_erred_retries_on_the_engine():
    """task-erred reports that do not err (svcretry_*): a retry or a stale run's report from the
    worker the task runs on, of a task something needs, is the reschedule's transitions on the
    engine (dgp_reschedule) followed by handle_task_erred's queue refill (dgp_release_tasks of
    nothing); no resync, every placement the engine's (validate=True)."""
    names = ["svcretry_c2var_sat1.1.npz", "svcretry_c2mini_satinf.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["resyncs"] == 0 and r["retries"] >= 40, r
        assert r["calls"]["erred_retries"] == r["retries"] == r["calls"]["reschedule"], r
        assert r["device_decisions"] == r["placements"], r


def test_extension_hands_back_on_unmodelled_events():
    """An engine without the event calls: the first such event ends GPU placement loudly
    ("not modelled") and the scheduler's own decisions carry on, equal to the reference's."""
    res = drive(EVENTS[:1], "--plain")
    assert not res[0]["active"] and "not modelled" in res[0]["reason"], res


def test_extension_hands_back_on_divergence():
    """A decision out of order: the extension detects it at once and the scheduler's own
    decide_worker carries on; the records are still the reference's."""
    res = drive(["c2var_sat1.1.npz", "c1_sat1.1.npz", "c3mini_sat1.1.npz"], "--diverge")
    for r in res:
        assert not r["active"] and "placement order differs" in r["reason"], r
        assert 0 < r["device_decisions"] < r["placements"], r


class NS:
    """A plain object with identity hashing, like TaskState / TaskGroup / TaskPrefix."""

    def __init__(self, **kw):
        self.worker_restrictions = self.host_restrictions = self.resource_restrictions = None
        self.__dict__.update(kw)


@pytest.fixture(params=["c", "python"])
def ingest(request, monkeypatch):
    """graph_from_tasks through the C pass (libdgpingest.so) and through the Python passes."""
    from distributed_amd import ext

    if request.param == "c" and ext._ingest_lib() is None:
        pytest.skip("libdgpingest.so not built")
    monkeypatch.setattr(ext, "_FORCE_PY_INGEST", request.param == "python")
    return request.param


def test_graph_from_tasks_layout(ingest):
    """graph_from_tasks on plain stand-ins (no dask needed): priority order, CSR, ids."""
    from distributed_amd.ext import graph_from_tasks

    P = {n: NS(name=n, duration_average=d) for n, d in (("a", -1.0), ("b", 0.5))}
    G = {n: NS(name=n) for n in ("a-1", "b-1")}
    t0 = NS(key="x", priority=(0, 1, 5), dependencies=[], prefix=P["a"], group=G["a-1"], who_wants=None, _rootish=None)
    t1 = NS(key="y", priority=(0, 1, 2), dependencies=[], prefix=P["a"], group=G["a-1"], who_wants=None, _rootish=True)
    t2 = NS(key="z", priority=(0, 1, 9), dependencies=[t0, t1], prefix=P["b"], group=G["b-1"], who_wants={1},
            _rootish=None)
    g, keys, prio = graph_from_tasks([t2, t0, t1], [1, 2])
    assert keys == ["y", "x", "z"] and prio == [(0, 1, 2), (0, 1, 5), (0, 1, 9)]
    assert g["dep_ptr"].tolist() == [0, 0, 0, 2] and g["dep_idx"].tolist() == [0, 1]
    assert g["prefix_names"] == ["a", "b"] and g["prefix_id"].tolist() == [0, 0, 1]
    assert g["prefix_default_dur"].tolist() == [-1.0, 0.5]
    assert g["group_prefix"].tolist() == [0, 1]
    assert g["wanted"].tolist() == [0, 0, 1] and g["rootish_override"].tolist() == [1, -1, -1]


def test_graph_from_tasks_c_pass_equals_python_passes(monkeypatch):
    """The C ingestion pass (csrc/dgp_ingest.c) and the Python passes give the same graph on
    random stand-ins: shuffled input order, shared prefixes / groups, dependencies on
    earlier tasks, wanted / _rootish / restricted rows."""
    from distributed_amd import ext

    if ext._ingest_lib() is None:
        pytest.skip("libdgpingest.so not built")
    rng = np.random.default_rng(4)
    P = [NS(name=f"p{i}", duration_average=float(i) - 1) for i in range(5)]
    G = [NS(name=f"g{i}", prefix=P[i % 5]) for i in range(12)]
    earlier = {f"old{i}": 100 + i for i in range(20)}
    olds = [NS(key=k) for k in earlier]
    tss = []
    for i in range(400):
        gi = int(rng.integers(12))
        deps = {tss[int(j)] for j in rng.integers(0, i, int(rng.integers(0, 5)))} if i else set()
        deps |= {olds[int(j)] for j in rng.integers(0, 20, int(rng.integers(0, 2)))}
        t = NS(key=f"t{i}", priority=(0, 1, i), dependencies=deps, prefix=G[gi].prefix, group=G[gi],
               who_wants={1} if rng.random() < 0.1 else None,
               _rootish=[None, True, False][int(rng.integers(3))],
               loose_restrictions=bool(rng.random() < 0.5))
        if rng.random() < 0.1:
            t.worker_restrictions = {f"w{int(rng.integers(8))}"}
        tss.append(t)
    order = [tss[int(i)] for i in rng.permutation(len(tss))]
    workers = [NS(address=f"w{i}") for i in range(8)]
    widx = {ws.address: i for i, ws in enumerate(workers)}

    def valid_workers(ts):
        return {ws for ws in workers if ws.address in ts.worker_restrictions}

    out = {}
    for mode in ("c", "python"):
        monkeypatch.setattr(ext, "_FORCE_PY_INGEST", mode == "python")
        out[mode] = ext.graph_from_tasks(order, [1] * 8, valid_workers, widx, earlier=earlier)
    (gc_, kc, pc), (gp, kp, pp) = out["c"], out["python"]
    assert kc == kp == [f"t{i}" for i in range(400)] and pc == pp
    assert set(gc_) == set(gp) and "restr_flags" in gc_
    for k in gc_:
        a, b = gc_[k], gp[k]
        assert (np.array_equal(a, b) if isinstance(a, np.ndarray) else a == b), k
    assert (gc_["dep_idx"] < 0).any()


def test_graph_from_tasks_names_earlier_tasks(ingest):
    """A later graph's dependency on an already uploaded task is named -1 - its engine index
    (dgp_add_graph); one outside both raises."""
    from distributed_amd.ext import graph_from_tasks

    P = NS(name="p", duration_average=0.1)
    G = NS(name="g")
    old = NS(key="old", priority=(0, 1, 0), dependencies=[], prefix=P, group=G, who_wants=None, _rootish=None)
    a = NS(key="a", priority=(0, 2, 1), dependencies=[old], prefix=P, group=G, who_wants=None, _rootish=None)
    b = NS(key="b", priority=(0, 2, 2), dependencies=[a, old], prefix=P, group=G, who_wants=None, _rootish=None)
    g, keys, _ = graph_from_tasks([b, a], [1], earlier={"old": 7})
    assert keys == ["a", "b"]
    assert g["dep_ptr"].tolist() == [0, 1, 3] and g["dep_idx"].tolist() == [-8, -8, 0]
    lost = NS(key="c", priority=(0, 2, 3), dependencies=[NS(key="zz")], prefix=P, group=G, who_wants=None,
              _rootish=None)
    with pytest.raises(ValueError, match="not in the uploaded graph"):
        graph_from_tasks([lost], [1], earlier={"old": 7})


def test_gpu_work_stealing_matches_reference_plugin():
    """GPUWorkStealing (distributed_amd/stealing.py) vs the reference WorkStealing on two
    identical states, two balance() calls each: request events, metrics, in-flight
    accounts, steal-request messages, bins and idle / saturated sets all equal
    (tests/steal_ext_driver.py; the engine is the oracle stand-in there). Before each
    balance() the incrementally kept task rows (StealRows) equal a full rebuild."""
    env = dict(os.environ, PYTHONHASHSEED="0")
    env.pop("PYTHONPATH", None)
    out = subprocess.run([PY39, os.path.join(REPO, "tests", "steal_ext_driver.py")], capture_output=True, text=True,
                         env=env, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    res = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(res) == 4
    for r in res:
        assert r["differ"] == [] and r["requests"] > 0 and r["rows_rebuilt"] == 0, r


def test_confirmed_steal_moves_the_task_on_the_engine():
    """The steal-response wrapper (plain stand-ins, no dask): a confirm that moved the task
    calls engine.move_task(task index, thief index); a reschedule hands placement back."""
    import asyncio
    from types import SimpleNamespace as NS

    from distributed_amd.ext import GPUPlacementExtension

    w0, w1 = NS(address="tcp://w0"), NS(address="tcp://w1")
    ts = NS(key="x", state="processing", processing_on=w0)
    moved = []

    class Stealing:
        async def move_task_confirm(self, *, key, state, stimulus_id, worker=None):
            t = sched.tasks[key]
            if state == "ready":  # the confirm branch (stealing.py:376-384)
                t.processing_on = w1
            else:  # the reschedule branch (:365-376)
                t.state = "released"
                t.processing_on = None

    class Engine:
        def move_task(self, t, w):
            moved.append((t, w))

    st = Stealing()
    sched = NS(tasks={"x": ts}, extensions={"stealing": st}, stream_handlers={"steal-response": st.move_task_confirm})
    ext = GPUPlacementExtension.__new__(GPUPlacementExtension)
    ext.scheduler, ext.active, ext.reason, ext.engine = sched, True, None, Engine()
    ext.task_index, ext.worker_index = {"x": 3}, {"tcp://w0": 0, "tcp://w1": 1}
    from collections import Counter, deque
    ext.stats, ext.pending = Counter(), deque()
    ext.suspended, ext._window = False, None
    ext._wrap_stealing()
    assert sched.stream_handlers["steal-response"] is st.move_task_confirm  # wrapped once, both places
    asyncio.run(sched.stream_handlers["steal-response"](key="x", state="ready", stimulus_id="s1", worker="tcp://w0"))
    assert moved == [(3, 1)] and ext.active and ext.stats["steals_confirmed"] == 1
    ts.processing_on = w0
    asyncio.run(sched.stream_handlers["steal-response"](key="x", state="executing", stimulus_id="s2"))
    assert moved == [(3, 1)] and not ext.active and "rescheduled" in ext.reason


def test_drop_ins_install_from_dask_config():
    """distributed.scheduler.gpu-placement.* (distributed_amd/config.py) in a real reference
    Scheduler, started: off by default (the reference's extensions untouched); installed by
    the ``distributed_amd.preload`` preload or by ``scheduler_extensions()`` as
    ``extensions=`` (scheduler.py:3890-3897's rule: GPUWorkStealing replaces WorkStealing,
    and no stealing at all when distributed.scheduler.work-stealing is off)."""
    env = dict(os.environ, PYTHONHASHSEED="0")
    env.pop("PYTHONPATH", None)
    out = subprocess.run([PY39, os.path.join(REPO, "tests", "config_driver.py")], capture_output=True, text=True,
                         env=env, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    res = {r["case"]: r for r in (json.loads(x) for x in out.stdout.splitlines() if x.startswith("{"))}
    d = res["default"]
    assert d["stealing"] == "WorkStealing" and d["placement"] == "NoneType" and "gpu-placement" not in d["extensions"]
    assert d["task_finished"] == "Scheduler.handle_task_finished"
    for c in ("preload", "extensions"):
        r = res[c]
        assert r["stealing"] == "GPUWorkStealing" and r["placement"] == "GPUPlacementExtension", r
        assert "WorkStealing" not in r["plugins"] and "GPUWorkStealing" in r["plugins"], r
        assert r["stealing_callback"] and r["task_finished"] == "GPUPlacementExtension.handle_task_finished", r
    n = res["no_stealing"]
    assert n["stealing"] is None and not n["stealing_callback"] and n["placement"] == "GPUPlacementExtension", n


def test_extension_compacts_the_prefix_table():
    """svcpfx_*: six later graphs with task prefixes of their own (75 over the stream, more
    than the engine's table of 32): the extension compacts the table to the live prefixes
    (prefixes.py; dgp_remap_prefixes + the dicts' resync) wherever a graph would not fit,
    stays active, and every placement comes from the engine (validate=True). Its remaps and
    resync rows equal the ones the generator recorded on the reference state, which the GPU
    test replays through the C ABI (tests/test_gpu_events.py)."""
    names = ["svcpfx_c2var_sat1.1.npz", "svcpfx_c2var_satinf.npz"]
    res = drive(names)
    assert [r["fixture"] for r in res] == names
    for r in res:
        assert r["active"] and r["device_decisions"] == r["placements"], r
        assert r["prefixes_seen"] > 64 and r["prefix_compactions"] >= 3, r
        assert r["remaps_checked"] == r["prefix_compactions"] and r["table"] <= 32, r
