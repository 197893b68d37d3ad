"""Wall time of the C2 replay only (GPU; A/B between builds): python tools/time_c2.py [reps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
g = graphs.random_dag(1_000_000, 1024, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
ts = []
for it in range(reps + 1):
    e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); ts.append(time.time() - t)
print(f"c2: {min(ts[1:]):.4f}s best of {reps} ({' '.join(f'{x:.4f}' for x in ts[1:])})", flush=True)
e.close()
