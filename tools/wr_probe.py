"""One C2-shaped replay (GPU), for PMC passes that vary the workload:
python tools/wr_probe.py N_TASKS N_WORKERS"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
n, w = int(sys.argv[1]), int(sys.argv[2])
g = graphs.random_dag(n, w, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
e.reset(); e.update_graph(); e.run_rounds(-1)
print("done", n, w, flush=True)
e.close()
