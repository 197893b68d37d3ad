"""Batch compute-task fields (tests/msg_model.py, the host-side model) on CPU: slices of a placement
log agree with the whole-log batch, every dependency's holder is the worker it was placed
on, and the reference's own messages are matched in tests/ext_driver.py (check_messages)."""
import numpy as np
import pytest

from distributed_amd import graphs
from msg_model import compute_task_batch, render_messages
from oracle import oracle

CFG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}


@pytest.fixture(scope="module")
def replay():
    g = graphs.random_dag(3000, 64, seed=4)
    return g, oracle.replay(g, CFG, snapshots=False)


def test_slices_match_whole_batch(replay):
    g, ref = replay
    n = len(ref["pl_task"])
    whole = compute_task_batch(g, ref["pl_task"], ref["pl_worker"], 0, n, g["nbytes"])
    placed_on = dict(zip(ref["pl_task"].tolist(), ref["pl_worker"].tolist()))
    assert all(placed_on[d] == h for d, h in zip(whole["dep_task"].tolist(), whole["dep_holder"].tolist()))
    assert np.array_equal(whole["dep_nbytes"], g["nbytes"][whole["dep_task"]])
    parts = [compute_task_batch(g, ref["pl_task"], ref["pl_worker"], a, min(700, n - a), g["nbytes"])
             for a in range(0, n, 700)]
    for k in ("task", "worker", "run_id", "dep_task", "dep_holder", "dep_nbytes"):
        assert np.array_equal(np.concatenate([p[k] for p in parts]), whole[k]), k


def test_render_and_errors(replay):
    g, ref = replay
    b = compute_task_batch(g, ref["pl_task"], ref["pl_worker"], 100, 5, g["nbytes"])
    keys = [f"t{i}" for i in range(g["n_tasks"])]
    msgs = render_messages(b, keys, [f"w{i}" for i in range(64)], lambda t: (0, 1, t), lambda t: 0.5)
    assert [m["key"] for m in msgs] == [keys[t] for t in ref["pl_task"][100:105]]
    for m, t in zip(msgs, ref["pl_task"][100:105]):
        deps = g["dep_idx"][g["dep_ptr"][t]:g["dep_ptr"][t + 1]]
        assert sorted(m["who_has"]) == sorted(keys[d] for d in deps) == sorted(m["nbytes"])
    with pytest.raises(ValueError):
        compute_task_batch(g, ref["pl_task"], ref["pl_worker"], len(ref["pl_task"]), 1, g["nbytes"])
    with pytest.raises(ValueError):  # a dependency placed after the batch window
        compute_task_batch(g, ref["pl_task"][::-1], ref["pl_worker"][::-1], 0, 10, g["nbytes"])


EV_FINISHED, EV_ADD_KEYS, EV_RELEASE_DATA = 0, 1, 2


@pytest.mark.parametrize("name", ["svcev_c2var_sat1.1", "svcev_c2mini_satinf", "svcev_dense_sat1.0"])
def test_replica_model_matches_recorded_messages(name):
    """The who_has / nbytes model the GPU test checks dgp_task_messages with (the completing
    worker, then add-keys adding and release-worker-data removing replicas) against the
    reference's own _task_to_msg messages (scheduler.py:3421-3450) recorded per placement
    by tests/golden/gen_service.py (tm_*)."""
    import os

    z = np.load(os.path.join(os.path.dirname(__file__), "golden", f"{name}.npz"), allow_pickle=False)
    dp, di = z["dep_ptr"], z["dep_idx"]
    stim = z["stim_nplaced"]
    pos = int(stim[0])
    first = int(z["tm_first"])
    who, nbytes = {}, {}
    checked = 0
    for i, (kd, t, w) in enumerate(zip(z["ev_kind"].tolist(), z["ev_task"].tolist(), z["ev_worker"].tolist())):
        if kd == EV_FINISHED:
            who[t], nbytes[t] = {w}, int(z["ev_nbytes"][i])
        elif kd == EV_ADD_KEYS:
            who.setdefault(t, set()).add(w)
        elif kd == EV_RELEASE_DATA:
            who[t].discard(w)
        for p in range(pos, pos + int(stim[i + 1])):
            r = p - first
            x = int(z["tm_task"][r])
            assert x == int(z["pl_task"][p])
            a = int(z["tm_dep_ptr"][r])
            for k, d in enumerate(di[dp[x]:dp[x + 1]].tolist()):
                assert int(z["tm_dep_task"][a + k]) == d
                hp = z["tm_hold_ptr"]
                assert z["tm_hold_idx"][hp[a + k]:hp[a + k + 1]].tolist() == sorted(who[d]), (i, x, d)
                assert int(z["tm_dep_nbytes"][a + k]) == nbytes[d]
                checked += 1
        pos += int(stim[i + 1])
    assert pos == len(z["pl_task"]) and checked > 3000
