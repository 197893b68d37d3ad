"""reset + update_graph alone on the C2 / C3 / C5 graphs (GPU; run under rocprofv3
--kernel-trace --stats for the per-kernel split): python tools/ug_time.py [reps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for name, g in (("c2", graphs.random_dag(1_000_000, 1024, seed=0)), ("c3", graphs.shuffle_graph(66_666, 512))):
    e = PlacementEngine(0)
    e.load(g, {"saturation": 1.1})
    ts, tu = [], []
    for it in range(reps + 1):
        t0 = time.perf_counter(); e.reset(); t1 = time.perf_counter(); e.update_graph(); t2 = time.perf_counter()
        ts.append(t1 - t0); tu.append(t2 - t1)
    print(f"{name}: reset {min(ts[1:]) * 1e3:.3f} ms, update_graph {min(tu[1:]) * 1e3:.3f} ms (best of {reps}), "
          f"placements {e.num_placements()}", flush=True)
    e.close()
