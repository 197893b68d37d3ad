"""One stream replay of C2-shaped work (diagnostic driver for profilers, GPU)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
g = graphs.random_dag(n, 1024, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
for it in range(2):
    e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); dt = time.time() - t
print(f"{n} tasks: {dt:.3f}s {e.num_placements() / dt / 1e6:.3f} M/s", flush=True)
