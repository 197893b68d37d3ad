"""Diagnostics: replay a svcwl_* stream through the engine, comparing the task states after
each loss event with the generator's (tests/golden/_dbg_<name>.npy, DGP_DEBUG_STATES=1)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_events as T
from oracle import oracle
from distributed_amd.engine import PlacementEngine
name = sys.argv[1]
path = os.path.join(T.GOLDEN, name + ".npz")
g, cfg, exp, meta = oracle.load_fixture(path)
z = np.load(path, allow_pickle=False)
dbg = np.load(os.path.join(T.GOLDEN, f"_dbg_{name}.npy"))
R = len(exp["round_nplaced"]) + 2
orig = PlacementEngine.lose_worker
k = [0]
def lose(self, w, p, h, order=(), killed=None):
    n = orig(self, w, p, h, order, killed)
    st = self.task_states()
    ref = dbg[k[0]]
    bad = np.flatnonzero(st != ref)
    print(f"loss {k[0]} worker {w} proc {list(map(int, p))} killed {killed} placed {n}: "
          f"{len(bad)} state mismatches {[(int(t), int(st[t]), int(ref[t])) for t in bad[:10]]}", flush=True)
    k[0] += 1
    return n
PlacementEngine.lose_worker = lose
otf = PlacementEngine.tasks_finished
def tf(self, t, w, *a):
    st = self.task_states()
    try:
        return otf(self, t, w, *a)
    except Exception:
        x = int(t[0])
        dp, di = g["dep_ptr"], g["dep_idx"]
        deps = di[dp[x]:dp[x + 1]].tolist()
        dents = np.flatnonzero([x in di[dp[y]:dp[y + 1]] for y in range(g["n_tasks"])]).tolist()
        print("FAILED completing", x, "on", list(map(int, w)), "state", int(st[x]), "deps", [(d, int(st[d])) for d in deps],
              "dependents", [(y, int(st[y]), [(d, int(st[d])) for d in di[dp[y]:dp[y + 1]].tolist()]) for y in dents], flush=True)
        raise
PlacementEngine.tasks_finished = tf
with PlacementEngine(0) as eng:
    eng.load(g, cfg, snapshots=R, results=False)
    eng.update_graph()
    try:
        T.drive_events(eng, g, z, exp)
    except Exception as e:
        print("ERROR", e)
