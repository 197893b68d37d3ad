"""The seam between the drop-in extension and the engine (verdict r02 item 8).

``distributed_amd/ext.py`` drives the engine through a handful of ``PlacementEngine``
methods. The extension tests run inside the reference scheduler with test doubles
(``tests/ext_driver.py``: ``FixtureEngine`` / ``EventEngine``, which serve a reference
fixture's decisions), because the GPU box has no dask and this container has no GPU. These
tests pin that the doubles and the real engine present the same interface:

* every engine method the extension calls exists on ``PlacementEngine`` and on the doubles
  it is driven with, with the same positional arity (the extension calls positionally);
* (GPU) the real engine returns what the extension consumes: ``placements()`` columns
  ``pl_task`` / ``pl_worker`` as int32 arrays of the requested length, ``tasks_finished()``
  a (int8 status per message, int) pair, the event calls the placement counts the
  extension adds to its queue, ``sync()`` the rows ``distributed_amd/sync.py`` builds.
"""
import ast
import inspect
import os
import re

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _ext_engine_calls():
    """Engine methods ext.py calls: ``self.engine.X(`` and the names it dispatches through
    ``_engine_op("X", ...)`` / ``_ENGINE_EVENTS``."""
    src = open(os.path.join(REPO, "distributed_amd", "ext.py")).read()
    names = set(re.findall(r"self\.engine\.([a-z_]+)\(", src))
    names |= set(re.findall(r'_engine_op\(\s*"([a-z_]+)"', src))
    m = re.search(r"_ENGINE_EVENTS = \(([^)]*)\)", src)
    names |= set(re.findall(r'"([a-z_]+)"', m.group(1)))
    return names


def _double_methods():
    """{class: {method: (n positional params without self, n required)}} of the doubles,
    read from tests/ext_driver.py without importing it (it imports the reference)."""
    tree = ast.parse(open(os.path.join(HERE, "ext_driver.py")).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name in ("FixtureEngine", "EventEngine", "GraphStimulusEngine"):
            ms = {}
            for f in node.body:
                if isinstance(f, ast.FunctionDef):
                    a = f.args
                    if a.vararg is not None:
                        ms[f.name] = None  # *args: any arity
                        continue
                    n = len(a.args) - 1
                    ms[f.name] = (n, n - len(a.defaults))
                elif isinstance(f, ast.Assign):  # aliases: sync_tasks = sync_workers = ...
                    for t in f.targets:
                        if isinstance(t, ast.Name) and isinstance(f.value, ast.Name):
                            ms[t.id] = ms.get(f.value.id)
            bases = [b.id for b in node.bases if isinstance(b, ast.Name)]
            for b in bases:
                for k, v in out.get(b, {}).items():
                    ms.setdefault(k, v)
            out[node.name] = ms
    return out


def test_extension_calls_exist_on_engine_and_doubles():
    from distributed_amd.engine import PlacementEngine

    calls = _ext_engine_calls()
    assert {"load", "update_graph", "tasks_finished", "placements", "num_placements", "add_worker", "add_graph",
            "remove_worker", "sync", "add_replicas", "task_erred"} <= calls, calls
    doubles = _double_methods()
    for name in sorted(calls):
        fn = getattr(PlacementEngine, name, None)
        assert fn is not None, f"PlacementEngine has no {name}()"
        ps = [p for p in inspect.signature(fn).parameters.values() if p.name != "self"
              and p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)]
        n_all = len(ps)
        n_req = sum(1 for p in ps if p.default is p.empty)
        # the double the extension is driven with in tests/test_ext.py: EventEngine covers all
        d = doubles["EventEngine"].get(name, "missing")
        if name == "graph_stimulus":  # EventEngine drives the resync path; this double runs the stimulus
            d = doubles["GraphStimulusEngine"].get(name, "missing")
        if name in ("move_task",):  # steal confirmations: tests/steal_ext_driver.py drives the real oracle
            continue
        assert d != "missing", f"EventEngine has no {name}()"
        if d is None:
            continue
        dn, dreq = d
        # the extension's positional calls must bind on both sides
        assert dreq <= n_all and n_req <= dn, (name, (n_req, n_all), (dreq, dn))


@pytest.mark.gpu
def test_engine_returns_what_the_extension_consumes():
    from distributed_amd import graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(600, 16, seed=9)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    with PlacementEngine(0) as eng:
        eng.load(g, cfg, results=False)  # the extension's load (ext.py update_graph)
        assert eng.update_graph() is None
        n = eng.num_placements()
        assert isinstance(n, int) and n > 0
        pl = eng.placements(0, n)  # ext.py _fetch
        for k in ("pl_task", "pl_worker"):
            assert pl[k].dtype == np.int32 and pl[k].shape == (n,), k
        t, w = int(pl["pl_task"][0]), int(pl["pl_worker"][0])
        # ext.py handle_task_finished_batch: columns from _message_fields, positional
        st, newp = eng.tasks_finished([t], [w], [0], [int(g["nbytes"][t])], [0.0], [0.01])
        assert isinstance(st, np.ndarray) and st.dtype == np.int8 and st.shape == (1,) and st[0] == 0
        assert isinstance(newp, int) and eng.num_placements() == n + newp
        more = eng.placements(n, newp)
        assert more["pl_task"].dtype == np.int32 and len(more["pl_task"]) == newp
        # the same through the resident kernel (the extension's mode): the placements of the
        # answer come from the mailbox, columns as the extension asks for them
        eng.set_resident(True)
        eng.set_task_messages(True)
        n1 = eng.num_placements()
        t2, w2 = int(pl["pl_task"][1]), int(pl["pl_worker"][1])  # still processing (run_id 1)
        st2, newp2 = eng.tasks_finished([t2], [w2], [1], [int(g["nbytes"][t2])], [0.0], [0.01])
        assert st2.dtype == np.int8 and st2.tolist() == [0] and isinstance(newp2, int)
        assert eng.num_placements() == n1 + newp2
        pr = eng.placements(n1, newp2, columns=("pl_task", "pl_worker"))
        assert set(pr) == {"pl_task", "pl_worker"} and pr["pl_task"].dtype == np.int32 and len(pr["pl_worker"]) == newp2
        # ext.py _fetch: the answer's compute-task message fields (from the mailbox)
        m = eng.task_messages(n1, newp2)
        assert m["dep_ptr"].dtype == np.int64 and len(m["dep_ptr"]) == newp2 + 1
        assert m["dep_task"].dtype == np.int32 and len(m["dep_task"]) == m["dep_ptr"][-1] == len(m["dep_nbytes"])
        assert m["holder_ptr"][-1] == len(m["holder_idx"])
        eng.set_resident(False)
        # event calls: the counts the extension's _fetch picks up afterwards
        assert eng.add_replicas([t], [(w + 1) % 16]) is None
        assert isinstance(eng.set_worker_status(3, 0), int)
        assert isinstance(eng.set_worker_status(3, 1), int)
        assert eng.heartbeat(100_000_000.0, [], []) is None
        assert isinstance(eng.add_worker(2), int)
        # a later independent graph (ext.py _add_graph: engine-wide prefix / group tables)
        g2 = graphs.random_dag(50, 17, seed=10)
        h = dict(g2, prio=g2["prio"] + len(g["prio"]), prefix_id=g2["prefix_id"], group_id=g2["group_id"] + len(
            g["group_prefix"]), prefix_default_dur=g["prefix_default_dur"],
            group_prefix=np.concatenate([g["group_prefix"], g2["group_prefix"]]))
        assert isinstance(eng.add_graph(h), int)
