"""Repeat the 1M replay; on failure print the pipeline post-mortem."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
n = int(sys.argv[1]); w = int(sys.argv[2]); reps = int(sys.argv[3])
g = graphs.random_dag(n, w, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
for it in range(reps):
    e.reset(); e.update_graph(); t = time.time()
    try:
        e.run_rounds(-1)
        print(f"rep {it}: ok {time.time() - t:.3f}s", flush=True)
    except Exception as ex:  # noqa: BLE001
        st = e.stats()
        print(f"rep {it}: FAIL {ex}", flush=True)
        print(" seq reg pre bld log ready busy gpend flags pred sid done walk rec qlen rend")
        print(" ", [st[f"wave_phase{i}"] for i in range(16)], flush=True)
        break
