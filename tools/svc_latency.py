"""Per-call cost of the service path (diagnostic): one dgp_tasks_finished per message on a
C2-shaped graph, with the engine's kernel timing on; prints the host time per call and the
stream kernel's device time per launch."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine

CFG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
g = graphs.random_dag(int(sys.argv[1]) if len(sys.argv) > 1 else 5000, int(sys.argv[2]) if len(sys.argv) > 2 else 1024, seed=5)
eng = PlacementEngine(0)
eng.load(g, CFG, results=False)
eng.update_graph()
eng.set_timing(True)
done, calls, t_call, t_fetch = 0, 0, 0.0, 0.0
while True:
    t0 = time.perf_counter()
    n = eng.num_placements()
    if n == done:
        break
    p = eng.placements(done, n - done)
    t_fetch += time.perf_counter() - t0
    t, w = p["pl_task"], p["pl_worker"]
    r = np.arange(done, n, dtype=np.int64)
    for i in range(min(len(t), int(os.environ.get("SVC_MAX_PER_ROUND", "1000000")))):
        t1 = time.perf_counter()
        eng.tasks_finished(t[i:i + 1], w[i:i + 1], r[i:i + 1], g["nbytes"][t[i:i + 1]], g["start"][t[i:i + 1]],
                           g["stop"][t[i:i + 1]])
        t_call += time.perf_counter() - t1
        calls += 1
    if os.environ.get("SVC_MAX_PER_ROUND") and len(t) > int(os.environ["SVC_MAX_PER_ROUND"]):
        k = int(os.environ["SVC_MAX_PER_ROUND"])
        eng.tasks_finished(t[k:], w[k:], r[k:], g["nbytes"][t[k:]], g["start"][t[k:]], g["stop"][t[k:]])
    done = n
    if calls >= int(os.environ.get("SVC_MAX_CALLS", "1000000000")):
        break
kt = eng.kernel_times()
print(f"calls {calls}: tasks_finished {t_call / calls * 1e6:.1f} us/call, fetch {t_fetch / calls * 1e6:.1f} us/call")
for k, (ms, nl) in kt.items():
    if nl:
        print(f"  {k}: {ms / nl * 1e3:.1f} us per launch x {nl}")
